"""In-tree build of every native artefact (no setuptools round trip, no JIT cache).

Artefacts (all land inside the package so gpurun snapshots carry them):

* ``kube_gpu_stats_amd/_kgs_native*.so`` – C++17 data plane (sampler threads,
  seqlocks, PMFW table reader, renderer, epoll HTTP) + pybind11 bindings; links
  ``libamd_smi``.
* ``kube_gpu_stats_amd/lib/libkgs_pmc_aql.so`` – the counter reader the exporter
  dlopens for ``--pmc aqlprofile`` (the default counter tier): aqlprofile PM4
  packets on a private AQL queue, pipelined and batched READs
  (``counters/pmc_aqlprofile.cpp``, ``include/kgs/aql_batch.h``, ``aql_ring.h``).
* ``kube_gpu_stats_amd/lib/libkgs_pmc.so`` – rocprofiler-sdk device-counting
  reader, a test-only cross-check (``--pmc rocprofiler`` needs
  ``KGS_PMC_CROSSCHECK=1``; it keeps one HSA helper thread spinning).
* ``kube_gpu_stats_amd/lib/libkgs_load.so`` – hand-written gfx950 HIP kernels
  (MFMA-bound, HBM-stream, xGMI peer copy) used as the synthetic load.

Rebuilds are incremental on source/header mtimes.  ``python -m
kube_gpu_stats_amd.native.build [--force]`` builds everything.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIB = os.path.join(PKG, "lib")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
OFFLOAD_ARCH = "gfx950"

CXXFLAGS = ["-std=c++17", "-O2", "-g1", "-fPIC", "-pthread", "-Wall", "-Wextra", "-Wno-unused-parameter",
            "-fvisibility=hidden"]


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def native_module_path() -> str:
    return os.path.join(PKG, "_kgs_native" + ext_suffix())


def pmc_lib_path() -> str:
    return os.path.join(LIB, "libkgs_pmc.so")


def pmc_aql_lib_path() -> str:
    return os.path.join(LIB, "libkgs_pmc_aql.so")


def load_lib_path() -> str:
    return os.path.join(LIB, "libkgs_load.so")


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _headers() -> list[str]:
    return sorted(glob.glob(os.path.join(HERE, "include", "kgs", "*.h")))


def metric_help_header() -> str:
    """Regenerate include/kgs/metric_help.h (the renderer's HELP / TYPE table) from the
    metric catalogue when the catalogue is newer; returns its path."""
    out = os.path.join(HERE, "include", "kgs", "metric_help.h")
    schema = os.path.join(PKG, "models", "schema.py")
    if _stale(out, [schema]):
        sys.path.insert(0, os.path.dirname(PKG))
        from kube_gpu_stats_amd.models.schema import cpp_header

        text = cpp_header()
        if not os.path.exists(out) or open(out).read() != text:
            with open(out + ".tmp", "w") as f:
                f.write(text)
            os.replace(out + ".tmp", out)
        else:
            os.utime(out)
    return out


def build_native(force: bool = False, verbose: bool = False) -> str:
    import pybind11

    metric_help_header()

    out = native_module_path()
    srcs = sorted(glob.glob(os.path.join(HERE, "src", "*.cpp")))
    if not force and not _stale(out, srcs + _headers() + [__file__]):
        return out
    objdir = os.path.join(HERE, "build", "obj")
    os.makedirs(objdir, exist_ok=True)
    inc = ["-I" + os.path.join(HERE, "include"), "-I" + pybind11.get_include(),
           "-I" + sysconfig.get_paths()["include"], "-I" + os.path.join(ROCM, "include")]

    def compile_one(src: str) -> str:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        if force or _stale(obj, [src] + _headers() + [__file__]):
            _run(["g++", *CXXFLAGS, *inc, "-c", src, "-o", obj], verbose)
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = f"{out}.{os.getpid()}.tmp"  # concurrent builders (one per rank) never share a temp file
    _run(["g++", "-shared", "-pthread", "-o", tmp, *objs, "-L" + os.path.join(ROCM, "lib"), "-lamd_smi",
          "-Wl,-rpath," + os.path.join(ROCM, "lib"), "-ldl", "-lz"], verbose)
    os.replace(tmp, out)
    return out


def build_pmc(force: bool = False, verbose: bool = False) -> str:
    out = pmc_lib_path()
    src = os.path.join(HERE, "counters", "pmc_rocprofiler.cpp")
    if not force and not _stale(out, [src, __file__]):
        return out
    os.makedirs(LIB, exist_ok=True)
    tmp = f"{out}.{os.getpid()}.tmp"  # concurrent builders (one per rank) never share a temp file
    _run(["g++", *CXXFLAGS, "-fvisibility=default", "-D__HIP_PLATFORM_AMD__=1", "-I" + os.path.join(ROCM, "include"), "-shared", src, "-o", tmp,
          "-L" + os.path.join(ROCM, "lib"), "-lrocprofiler-sdk", "-lhsa-runtime64",
          "-Wl,-rpath," + os.path.join(ROCM, "lib")], verbose)
    os.replace(tmp, out)
    return out


def build_pmc_aql(force: bool = False, verbose: bool = False) -> str:
    """Direct CP counter reader over aqlprofile (no profiler framework, no spinning helper thread)."""
    out = pmc_aql_lib_path()
    src = os.path.join(HERE, "counters", "pmc_aqlprofile.cpp")
    deps = [src, os.path.join(HERE, "include", "kgs", "aql_ring.h"), os.path.join(HERE, "include", "kgs", "aql_batch.h"),
            os.path.join(HERE, "include", "kgs", "aql_ib.h"),
            __file__]
    if not force and not _stale(out, deps):
        return out
    os.makedirs(LIB, exist_ok=True)
    tmp = f"{out}.{os.getpid()}.tmp"
    _run(["g++", *CXXFLAGS, "-fvisibility=default", "-D__HIP_PLATFORM_AMD__=1", "-I" + os.path.join(ROCM, "include"),
          "-I" + os.path.join(HERE, "include"),
          "-shared", src, "-o", tmp, "-L" + os.path.join(ROCM, "lib"), "-lhsa-runtime64", "-lhsa-amd-aqlprofile64",
          "-Wl,-rpath," + os.path.join(ROCM, "lib")], verbose)
    os.replace(tmp, out)
    return out


def build_load(force: bool = False, verbose: bool = False) -> str:
    out = load_lib_path()
    src = os.path.join(PKG, "ops", "hip", "load_kernels.hip")
    if not force and not _stale(out, [src, __file__]):
        return out
    os.makedirs(LIB, exist_ok=True)
    tmp = f"{out}.{os.getpid()}.tmp"  # concurrent builders (one per rank) never share a temp file
    _run([os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={OFFLOAD_ARCH}", "-O3", "-std=c++17", "-fPIC",
          "-shared", src, "-o", tmp], verbose)
    os.replace(tmp, out)
    return out


def build_tsan_test(verbose: bool = False, sanitizer: str = "thread") -> str:
    """Host-only test of the seqlock / ring / sampler under a sanitizer
    (``thread``, or ``address,undefined``).  Objects compile in parallel."""
    tag = "tsan" if sanitizer == "thread" else "asan"
    out = os.path.join(HERE, "build", f"test_core_{tag}")
    srcs = [os.path.join(HERE, "tests", "test_core.cpp")] + [
        os.path.join(HERE, "src", f) for f in ("sampler.cpp", "backend_mock.cpp", "pmc.cpp", "gpu_metrics.cpp", "util.cpp",
                                              "exporter.cpp", "render.cpp", "http.cpp", "backend_amdsmi.cpp",
                                              "kfd_procs.cpp")]
    objdir = os.path.join(HERE, "build", f"obj_{tag}")
    os.makedirs(objdir, exist_ok=True)
    metric_help_header()
    flags = ["-std=c++17", "-O1", "-g", f"-fsanitize={sanitizer}", "-fno-omit-frame-pointer", "-pthread"]
    if _stale(out, srcs + _headers() + [__file__]):
        def compile_one(src: str) -> str:
            obj = os.path.join(objdir, os.path.basename(src) + ".o")
            if _stale(obj, [src] + _headers() + [__file__]):
                _run(["g++", *flags, "-I" + os.path.join(HERE, "include"), "-I" + os.path.join(ROCM, "include"),
                      "-c", src, "-o", obj], verbose)
            return obj

        with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
            objs = list(ex.map(compile_one, srcs))
        tmp = f"{out}.{os.getpid()}.tmp"
        _run(["g++", *flags, *objs, "-o", tmp, "-L" + os.path.join(ROCM, "lib"), "-lamd_smi",
              "-Wl,-rpath," + os.path.join(ROCM, "lib"), "-ldl", "-lz"], verbose)
        os.replace(tmp, out)
    return out


def build_all(force: bool = False, verbose: bool = False, hip: bool = True) -> dict:
    res = {"native": build_native(force, verbose)}
    try:
        res["pmc"] = build_pmc(force, verbose)
        res["pmc_aql"] = build_pmc_aql(force, verbose)
    except RuntimeError as e:  # ROCm profiling headers missing on a host-only image
        res["pmc_error"] = str(e)
    if hip:
        res["load"] = build_load(force, verbose)
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--no-hip", action="store_true")
    a = ap.parse_args(argv)
    res = build_all(a.force, a.verbose, hip=not a.no_hip)
    for k, v in res.items():
        print(f"{k}: {v}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
