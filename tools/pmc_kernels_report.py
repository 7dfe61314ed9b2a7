"""Counters per kernel from the rocprofv3 --pmc passes of tools/pmc_kernels.py vs the known work."""

import sys as _sys

if __name__ == "__main__" and {"-h", "--help"} & set(_sys.argv[1:]):
    print(__doc__)  # a one-off GPU probe: no flags beyond this
    _sys.exit(0)
import csv
import glob
import json
import sys

root = sys.argv[1]
work = {}
for line in open(f"{root}/work.log"):
    if line.startswith("{"):
        work = json.loads(line)
per: dict = {}
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        k = "mfma" if "mfma_bf16" in name else "triad" if "triad_f32" in name else "copy" if "copy_f32" in name else None
        if k is None:
            continue
        d = per.setdefault(k, {}).setdefault(r["Counter_Name"], [])
        d.append(float(r["Counter_Value"]))
mean = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
out = ["| kernel | counter | mean per dispatch | known work | ratio |", "|---|---|---|---|---|"]
m = mean.get("mfma", {})
if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in m:
    flops = m["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512
    out.append(f"| mfma_bf16 | MFMA_MOPS_BF16 × 512 | {flops:.4g} FLOP | {work['mfma_flops']:.4g} FLOP | "
               f"{flops / work['mfma_flops']:.4f} |")
if "MfmaUtil" in m:
    out.append(f"| mfma_bf16 | MfmaUtil | {m['MfmaUtil']:.1f} % | — | — |")
for k, key in (("triad", "triad_bytes"), ("copy", "copy_bytes")):
    t = mean.get(k, {})
    if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
        moved = (t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024
        out.append(f"| {k} | FETCH_SIZE + WRITE_SIZE | {moved:.4g} B | {work[key]:.4g} B | {moved / work[key]:.4f} |")
if work:
    out.append("")
    out.append(f"Timed with HIP events in the same process: MFMA {work['mfma_flops'] / work['mfma_ms'] / 1e9:.0f} TFLOP/s, "
               f"triad {work['triad_bytes'] / work['triad_ms'] / 1e9:.2f} TB/s.")
print("\n".join(out))
print(json.dumps(mean))
