// Direct reader of the PMFW metrics table (`/sys/class/drm/cardN/device/gpu_metrics`).
//
// On MI355X (gfx950) the kernel exposes format 1 / content 8 (3872 bytes).  One
// pread of the table costs ≈46 µs on the box versus ≈270 µs through
// amdsmi_get_gpu_metrics_info (measured, profiles/probe_summary.md), so the fast
// tier parses the table itself.  Field offsets were verified against a live
// table (tests/test_gpu_metrics.py pins them with a captured MI355X blob).
#pragma once

#include <cstddef>
#include <cstdint>

#include "kgs/sample.h"

namespace kgs {

constexpr size_t kGpuMetricsV18Size = 3872;
constexpr int kV18NumXcp = 8;

// Parse a v1.8 table into `out` (fields not in the table are left untouched).
// Returns 0 on success, -1 on bad header / size.
int parse_gpu_metrics_v1_8(const uint8_t* buf, size_t len, GpuSample& out);

// Header peek: returns (format << 8) | content, or -1.
int gpu_metrics_revision(const uint8_t* buf, size_t len);

// MI355X compute partitioning (DPX / QPX / CPX) makes each partition its own
// device — own KFD node, DRM card, HSA agent and device-plugin ID — over the
// SAME PCI function and therefore the same PMFW table, which lists the XCCs of
// every partition in order.  Partition p of an n-way split owns XCCs
// [p·8/n, (p+1)·8/n).  This rewrites a chip-wide sample as that partition's
// view: per-XCC arrays shifted to the owned XCCs, gfx busy (instantaneous and
// accumulated) the mean over them.  UMC, power, thermals and xGMI stay
// chip-wide (the firmware does not split them).  No-op for an SPX device.
void restrict_to_xccs(GpuSample& s, uint32_t first, uint32_t count);

// Number of compute partitions of a mode name: SPX 1, DPX 2, QPX 4, CPX 8 (unknown → 1).
uint32_t partitions_of_mode(const char* mode);

}  // namespace kgs
