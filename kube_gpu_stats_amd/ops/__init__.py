"""Hand-written gfx950 HIP kernels (synthetic load for the overhead benchmark)."""
