"""Python handle on the gfx950 synthetic-load kernels (``ops/hip/load_kernels.hip``).

The kernels are the calibrated yardstick for the exporter's GPU-time overhead
(SURVEY.md §7.4.3): their throughput is measured with the sampler off and on, on
the same device, in the same process.  Memory comes from PyTorch (HIP caching
allocator) and launches go on the current torch stream, so the bench can bracket
them with ``torch.cuda.synchronize``.

There is deliberately no eager-PyTorch fallback: on a GPU box the HIP library
must load, or these functions raise.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

from ..native import build as _build

_LIB: ctypes.CDLL | None = None
BLOCK = 256
WAVES_PER_BLOCK = BLOCK // 64
MFMA_FLOP_PER_WAVE_ITER = 4 * 2 * 16 * 16 * 32  # four 16x16x32 MFMAs


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = _build.load_lib_path()
        if not os.path.exists(path):
            _build.build_load()
        L = ctypes.CDLL(path)
        L.kgs_load_last_error.restype = ctypes.c_char_p
        L.kgs_load_mfma_bf16.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_void_p]
        L.kgs_load_mfma_bf16_xcc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
        L.kgs_load_triad_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                         ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        L.kgs_load_triad_f32_xcc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                             ctypes.c_size_t, ctypes.c_int, ctypes.c_uint, ctypes.c_void_p]
        L.kgs_load_triad_f32_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                            ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.kgs_load_copy_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_void_p]
        L.kgs_load_enable_peer.argtypes = [ctypes.c_int, ctypes.c_int]
        L.kgs_load_gather64.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.kgs_load_reread.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]
        _LIB = L
    return _LIB


def _check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError(lib().kgs_load_last_error().decode())


def _stream_ptr(stream=None) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def mfma_bf16(A, B, C, nblocks: int, iters: int, stream=None) -> None:
    """C[w] = iters · (A @ B) for every wave w; A [16,32] bf16, B [32,64] bf16, C [nblocks*4,16,64] f32."""
    import torch

    assert A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16 and C.dtype == torch.float32
    assert tuple(A.shape) == (16, 32) and tuple(B.shape) == (32, 64), (A.shape, B.shape)
    assert A.is_contiguous() and B.is_contiguous() and C.is_contiguous()
    assert C.numel() >= nblocks * WAVES_PER_BLOCK * 16 * 64, "C too small for the grid"
    assert A.device == B.device == C.device and A.is_cuda
    _check(lib().kgs_load_mfma_bf16(A.data_ptr(), B.data_ptr(), C.data_ptr(), int(nblocks), int(iters),
                                    _stream_ptr(stream)))


def mfma_bf16_xcc(A, B, C, nblocks: int, iters: int, xcc_mask: int, xcc_out=None, stream=None) -> None:
    """mfma_bf16 on the XCDs in ``xcc_mask`` only: a workgroup whose hardware XCC id
    (HW_REG_XCC_ID) is not in the mask skips the loop and writes zeros.  ``xcc_out``
    (int32 [nblocks], optional) receives every workgroup's XCC id."""
    import torch

    assert A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16 and C.dtype == torch.float32
    assert tuple(A.shape) == (16, 32) and tuple(B.shape) == (32, 64), (A.shape, B.shape)
    assert A.is_contiguous() and B.is_contiguous() and C.is_contiguous()
    assert C.numel() >= nblocks * WAVES_PER_BLOCK * 16 * 64, "C too small for the grid"
    assert A.device == B.device == C.device and A.is_cuda
    out_ptr = 0
    if xcc_out is not None:
        assert xcc_out.dtype == torch.int32 and xcc_out.numel() >= nblocks and xcc_out.device == A.device
        out_ptr = xcc_out.data_ptr()
    _check(lib().kgs_load_mfma_bf16_xcc(A.data_ptr(), B.data_ptr(), C.data_ptr(), int(nblocks), int(iters),
                                        int(xcc_mask) & 0xFFFF, out_ptr, _stream_ptr(stream)))


def triad_f32(a, b, c, s: float, nblocks: int = 0, stream=None, nt: bool = True) -> None:
    """c = a + s·b over float32 vectors (length multiple of 4)."""
    import torch

    n = a.numel()
    assert a.dtype == b.dtype == c.dtype == torch.float32 and b.numel() == n and c.numel() >= n and n % 4 == 0
    assert a.is_contiguous() and b.is_contiguous() and c.is_contiguous()
    for t in (a, b, c):
        assert t.data_ptr() % 16 == 0
    if nblocks <= 0:
        nblocks = default_stream_blocks(n)
    _check(lib().kgs_load_triad_f32_ex(a.data_ptr(), b.data_ptr(), c.data_ptr(), float(s), n, int(nblocks),
                                       int(bool(nt)), _stream_ptr(stream)))


def triad_f32_xcc(a, b, c, s: float, xcc_mask: int, nblocks: int = 0, stream=None) -> None:
    """triad_f32 on the XCDs in ``xcc_mask`` only (hardware XCC id); elements owned by
    workgroups on other XCDs are left untouched."""
    import torch

    assert a.dtype == b.dtype == c.dtype == torch.float32 and a.numel() == b.numel() == c.numel()
    assert a.numel() % 4 == 0 and a.is_cuda and a.is_contiguous() and b.is_contiguous() and c.is_contiguous()
    nb = nblocks or default_stream_blocks(a.numel())
    _check(lib().kgs_load_triad_f32_xcc(a.data_ptr(), b.data_ptr(), c.data_ptr(), float(s), a.numel(), nb,
                                        int(xcc_mask) & 0xFFFF, _stream_ptr(stream)))


def copy_f32(src, dst, nblocks: int = 0, stream=None) -> None:
    """dst = src (src may live on a peer GPU after enable_peer)."""
    import torch

    n = src.numel()
    assert src.dtype == dst.dtype == torch.float32 and dst.numel() >= n and n % 4 == 0
    assert src.data_ptr() % 16 == 0 and dst.data_ptr() % 16 == 0
    if nblocks <= 0:
        nblocks = default_stream_blocks(n)
    _check(lib().kgs_load_copy_f32(src.data_ptr(), dst.data_ptr(), n, int(nblocks), _stream_ptr(stream)))


def gather64(src, nlines: int, per_thread: int, seed: int, out, shift: int = 3, stream=None) -> None:
    """out[t] = Σ of the 16 floats of each of `per_thread` random 64 B lines of `src`
    (line = (x >> shift) & (nlines-1), x the 32-bit LCG of gather64_ref); nlines a
    power of two, src ≥ nlines·16 floats, out = nblocks·256 floats."""
    import torch

    assert src.dtype == out.dtype == torch.float32 and src.is_contiguous() and out.is_contiguous()
    assert nlines > 0 and nlines & (nlines - 1) == 0 and src.numel() >= nlines * 16 and src.data_ptr() % 16 == 0
    assert out.numel() % BLOCK == 0 and 0 <= shift <= 31 and src.device == out.device
    _check(lib().kgs_load_gather64(src.data_ptr(), nlines, shift, int(per_thread), int(seed) & 0xFFFFFFFF,
                                   out.numel() // BLOCK, out.data_ptr(), _stream_ptr(stream)))


def gather64_ref(src, nlines: int, per_thread: int, seed: int, threads, shift: int = 3):
    """fp32 torch reference of gather64 for the thread ids in `threads` (int64 tensor)."""
    import torch

    M = 0xFFFFFFFF
    x = (seed ^ ((threads * 2654435761) & M)) & M
    lines = src.view(-1, 16)
    acc = torch.zeros(threads.numel(), dtype=torch.float32, device=src.device)
    for _ in range(per_thread):
        x = (x * 1664525 + 1013904223) & M
        acc += lines[((x >> shift) & (nlines - 1)).to(src.device)].sum(-1)
    return acc


def reread(src, passes: int, out, stream=None) -> None:
    """out[t] = passes × Σ_k src4[t + k·T] (summed as float4 lanes), T = out.numel()."""
    import torch

    assert src.dtype == out.dtype == torch.float32 and src.is_contiguous() and out.is_contiguous()
    assert src.numel() % 4 == 0 and out.numel() % BLOCK == 0 and src.data_ptr() % 16 == 0 and src.device == out.device
    _check(lib().kgs_load_reread(src.data_ptr(), src.numel(), int(passes), out.numel() // BLOCK, out.data_ptr(),
                                 _stream_ptr(stream)))


def enable_peer(dev: int, peer: int) -> None:
    _check(lib().kgs_load_enable_peer(int(dev), int(peer)))


def default_stream_blocks(n: int, cus: int = 256) -> int:
    # 32 contiguous chunks per CU (8192 blocks: best of 1k-16k measured), but at
    # least 4 float4 per thread so every lane runs a full unrolled trip.
    return max(1, min(cus * 32, n // (4 * 4 * BLOCK)))


@dataclass
class LoadStep:
    """One benchmark step of mixed synthetic load on one GPU.

    ``mfma_iters`` MFMA iterations on a full grid followed by one HBM triad over
    ``stream_bytes`` of float32 (three arrays), on the current torch stream.
    """

    device: int = 0
    mfma_blocks: int = 2048
    mfma_iters: int = 4096
    stream_bytes: int = 3 << 30

    def __post_init__(self):
        import torch

        dev = torch.device("cuda", self.device)
        g = torch.Generator(device="cpu").manual_seed(1234)
        self.A = torch.randn(16, 32, generator=g).to(torch.bfloat16).to(dev)
        self.B = torch.randn(32, 64, generator=g).to(torch.bfloat16).to(dev)
        self.C = torch.empty(self.mfma_blocks * WAVES_PER_BLOCK * 16 * 64, dtype=torch.float32, device=dev)
        n = (self.stream_bytes // 12) // 4 * 4
        self.a = torch.rand(n, dtype=torch.float32, device=dev)
        self.b = torch.rand(n, dtype=torch.float32, device=dev)
        self.c = torch.empty(n, dtype=torch.float32, device=dev)
        self.n = n

    @property
    def flops(self) -> float:
        return float(self.mfma_blocks * WAVES_PER_BLOCK * self.mfma_iters * MFMA_FLOP_PER_WAVE_ITER)

    @property
    def bytes(self) -> float:
        return float(self.n * 12)

    def run_mfma(self) -> None:
        mfma_bf16(self.A, self.B, self.C, self.mfma_blocks, self.mfma_iters)

    def run_stream(self) -> None:
        triad_f32(self.a, self.b, self.c, 1.5)

    def __call__(self) -> None:
        self.run_mfma()
        self.run_stream()
