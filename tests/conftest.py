import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def gpurun_out_digest() -> str:
    """sha256 over every file under gpurun_out/ (path, size, bytes)."""
    import hashlib

    h = hashlib.sha256()
    root = os.path.join(REPO, "gpurun_out")
    for d, dirs, files in sorted(os.walk(root)):
        dirs.sort()
        for f in sorted(files):
            if d == root and f == ".last_call.json":
                continue  # the gpurun client's own record of its last call, not a test's output
            p = os.path.join(d, f)
            h.update(os.path.relpath(p, root).encode())
            try:
                with open(p, "rb") as fh:
                    h.update(fh.read())
            except OSError:
                h.update(b"<unreadable>")
    return h.hexdigest()


GPURUN_OUT_AT_START = gpurun_out_digest()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on a GPU box)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds")


@pytest.fixture(scope="session")
def N():
    """The compiled native data plane (built in-tree on first use)."""
    from kube_gpu_stats_amd import load_native

    return load_native()


@pytest.fixture
def mock_exporter(N):
    made = []

    def make(**kw):
        cfg = {"backend": "mock", "mock": {"n_gpus": kw.pop("n_gpus", 4)}, "hz": kw.pop("hz", 100), "port": 0,
               "node_name": "node-a", "pin_numa": False}
        if "mock" in kw:
            cfg["mock"].update(kw.pop("mock"))
        cfg.update(kw)
        ex = N.Exporter(cfg)
        ex.start()
        made.append(ex)
        return ex

    yield make
    for ex in made:
        ex.stop()
