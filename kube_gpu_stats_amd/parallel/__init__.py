"""Device fan-out, xGMI topology and the one-process-per-GPU bench helpers.

The exporter's parallel axis is *device fan-out*: one native sampler thread per
GPU (native/src/sampler.cpp), pinned to the GPU's NUMA node, merged at scrape
time.  ``topology`` discovers the xGMI mesh; ``dist`` holds the
torchrun/RCCL helpers the benchmark uses.
"""
