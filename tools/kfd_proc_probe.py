"""Where does per-process CU occupancy come from, and why does AMD SMI print
"Unable to open queues directory for process N" ?

With a HIP context open in this process (torch on cuda:0), dump what the KFD exposes
under /sys/class/kfd/kfd/proc/<pid>/ for every listed process (file names, small file
contents, which opens fail and with what errno), this process's PID-namespace view
(/proc/self/status NSpid), and what amdsmi_get_gpu_process_list returns — with fd 1 and
fd 2 captured separately around the call, so the message's stream and PID are known.

    python tools/kfd_proc_probe.py --out gpurun_out/kfd_proc.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile


def walk(path: str, depth: int = 0) -> dict:
    out: dict = {}
    try:
        names = sorted(os.listdir(path))
    except OSError as e:
        return {"<error>": f"{type(e).__name__}: {e}"}
    for n in names:
        p = os.path.join(path, n)
        if os.path.isdir(p) and not os.path.islink(p):
            out[n + "/"] = walk(p, depth + 1) if depth < 2 else "<dir>"
        else:
            try:
                with open(p) as f:
                    out[n] = f.read(200).strip()
            except OSError as e:
                out[n] = f"<{type(e).__name__}: errno {e.errno}>"
    return out


def capture(fn):
    """Run fn() with fd 1 and fd 2 redirected to temp files; return (result, stdout, stderr)."""
    sys.stdout.flush()
    sys.stderr.flush()
    saved = os.dup(1), os.dup(2)
    f1, f2 = tempfile.TemporaryFile(), tempfile.TemporaryFile()
    os.dup2(f1.fileno(), 1)
    os.dup2(f2.fileno(), 2)
    try:
        res = fn()
    finally:
        os.dup2(saved[0], 1)
        os.dup2(saved[1], 2)
        os.close(saved[0])
        os.close(saved[1])
    f1.seek(0)
    f2.seek(0)
    return res, f1.read().decode(errors="replace"), f2.read().decode(errors="replace")


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--out", default="gpurun_out/kfd_proc.json")
    a = ap.parse_args()
    import torch

    x = torch.ones(1 << 20, device="cuda:0")
    torch.cuda.synchronize()
    rep: dict = {"self_pid": os.getpid()}
    try:
        with open("/proc/self/status") as f:
            rep["nspid"] = [ln.split()[1:] for ln in f if ln.startswith("NSpid")]
    except OSError as e:
        rep["nspid"] = str(e)
    root = "/sys/class/kfd/kfd/proc"
    rep["kfd_proc"] = walk(root)
    rep["topology_gpu_ids"] = {}
    for node in sorted(os.listdir("/sys/class/kfd/kfd/topology/nodes")):
        try:
            with open(f"/sys/class/kfd/kfd/topology/nodes/{node}/gpu_id") as f:
                rep["topology_gpu_ids"][node] = f.read().strip()
        except OSError:
            pass
    try:
        import amdsmi

        amdsmi.amdsmi_init()
        h = amdsmi.amdsmi_get_processor_handles()[0]

        def plist():
            return amdsmi.amdsmi_get_gpu_process_list(h)

        procs, out, err = capture(plist)
        rep["amdsmi_process_list"] = [{k: (str(v) if not isinstance(v, (int, float, str)) else v)
                                       for k, v in (p.items() if isinstance(p, dict) else {"p": p}.items())}
                                      for p in procs]
        rep["amdsmi_stdout"] = out[-2000:]
        rep["amdsmi_stderr"] = err[-2000:]
        amdsmi.amdsmi_shut_down()
    except Exception as e:  # noqa: BLE001
        rep["amdsmi_error"] = f"{type(e).__name__}: {e}"
    del x
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rep, f, indent=1)
    print(json.dumps({k: rep[k] for k in ("self_pid", "nspid")}))
    print(json.dumps(rep.get("amdsmi_stdout", ""))[:500], json.dumps(rep.get("amdsmi_stderr", ""))[:500])
    return 0


if __name__ == "__main__":
    sys.exit(main())
