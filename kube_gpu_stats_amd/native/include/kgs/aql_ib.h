// Lite READ indirect buffer (--pmc-lite, native/counters/pmc_aqlprofile.cpp).
//
// aqlprofile's READ IB (profiles/r1/lean/read_packet_dump_base.txt) is one
// PRED_EXEC region per XCC.  Inside each: GRBM_GFX_INDEX = broadcast, the GRBM /
// CP counters' COPY_DATA register→memory packets, then per shader engine a
// GRBM_GFX_INDEX write selecting that SE followed by the SQ (and, in the full
// set, TA) counters' copies.  What a READ costs a stream of µs kernels grows with
// its packets (profiles/r4/ r4h: 3.84 % at 8 kHz for the base set's 56 results,
// 2.39 % for the 24 of `--pmc-set util`, a fixed ≈1.3 % per READ the rest), and
// NOP-ing the per-SE copies in place saved little (3.56 %): the CP still fetches
// and decodes every packet.  So a lite READ's IB is a compacted copy without the
// per-SE sections: each GRBM_GFX_INDEX write that selects one SE, together with
// the COPY_DATA→memory packets after it, is dropped when nothing else follows
// before the next GRBM_GFX_INDEX write or the end of the enclosing PRED_EXEC
// region; type-3 NOPs (left by the lean rewrite) are dropped too.  PRED_EXEC exec
// counts shrink by what their region lost; every other packet is copied verbatim
// (their addresses are absolute).  The copy is validated before use — it must
// re-parse into whole packets, every PRED_EXEC region must end on a packet
// boundary, and its COPY_DATA destinations must be the input's minus the dropped
// ones, in order — and the reader keeps the full IB for the slot otherwise.
//
// Pure functions on dword arrays, header-only, unit-tested without a GPU
// (native/tests/test_core.cpp).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace kgs {

constexpr uint32_t kPm4Nop = 0x10, kPm4PredExec = 0x23, kPm4CopyData = 0x40, kPm4SetUconfigReg = 0x79;
constexpr uint32_t kGrbmGfxIndexReg = 0x200;      // SET_UCONFIG_REG offset of GRBM_GFX_INDEX
constexpr uint32_t kGrbmSeBroadcast = 1u << 31;   // GRBM_GFX_INDEX.SE_BROADCAST_WRITES
constexpr uint32_t kPredExecCountMask = 0x3FFF;   // PRED_EXEC: dwords predicated after the packet

inline uint32_t pm4_type(uint32_t h) { return h >> 30; }
inline uint32_t pm4_op(uint32_t h) { return (h >> 8) & 0xFF; }
inline uint32_t pm4_len(uint32_t h) { return ((h >> 16) & 0x3FFF) + 2; }  // dwords, header included

// COPY_DATA with dst_sel = memory (5): a counter result landing in the output buffer.
inline bool pm4_copy_to_mem(const uint32_t* p) {
  return pm4_op(p[0]) == kPm4CopyData && pm4_len(p[0]) == 6 && ((p[1] >> 8) & 0xF) == 5;
}
// Bytes one COPY_DATA writes: COUNT_SEL (control bit 16) selects 64 bits, else 32.
inline uint32_t pm4_copy_bytes(const uint32_t* p) { return (p[1] >> 16) & 1u ? 8u : 4u; }
inline uint64_t pm4_copy_dst(const uint32_t* p) {
  return (static_cast<uint64_t>(p[4]) | (static_cast<uint64_t>(p[5]) << 32)) & ~3ull;
}
// SET_UCONFIG_REG of GRBM_GFX_INDEX alone; *se_select = it selects one SE.
inline bool pm4_gfx_index(const uint32_t* p, bool* se_select) {
  if (pm4_op(p[0]) != kPm4SetUconfigReg || pm4_len(p[0]) != 3 || p[1] != kGrbmGfxIndexReg) return false;
  *se_select = !(p[2] & kGrbmSeBroadcast);
  return true;
}

// The COPY_DATA→memory destinations of an IB, in order; false if it does not parse
// into whole type-3 packets (type-2 fillers allowed) with PRED_EXEC regions ending
// on packet boundaries.
inline bool ib_copy_dsts(const uint32_t* ib, uint32_t ndw, std::vector<uint64_t>* dsts, std::string* why = nullptr) {
  uint32_t region_end = 0;  // 0 = not inside a PRED_EXEC region
  for (uint32_t i = 0; i < ndw;) {
    if (region_end && i == region_end) region_end = 0;
    if (region_end && i > region_end) {
      if (why) *why = "PRED_EXEC region ends inside a packet at dword " + std::to_string(region_end);
      return false;
    }
    const uint32_t h = ib[i];
    if (pm4_type(h) == 2) { ++i; continue; }
    if (pm4_type(h) != 3) {
      if (why) *why = "non type-3 header at dword " + std::to_string(i);
      return false;
    }
    const uint32_t len = pm4_len(h);
    if (i + len > ndw) {
      if (why) *why = "packet runs past the IB at dword " + std::to_string(i);
      return false;
    }
    if (pm4_op(h) == kPm4PredExec) {
      if (region_end) {
        if (why) *why = "nested PRED_EXEC at dword " + std::to_string(i);
        return false;
      }
      region_end = i + len + (ib[i + 1] & kPredExecCountMask);
      if (region_end > ndw) {
        if (why) *why = "PRED_EXEC region runs past the IB at dword " + std::to_string(i);
        return false;
      }
    } else if (pm4_copy_to_mem(ib + i) && dsts) {
      dsts->push_back(pm4_copy_dst(ib + i));
    }
    i += len;
  }
  if (region_end && region_end != ndw) {
    if (why) *why = "PRED_EXEC region open at the end";
    return false;
  }
  return true;
}

struct IbCompact {
  bool ok = false;
  uint32_t dropped_copies = 0;  // per-SE COPY_DATA packets left out
  uint32_t dropped_dw = 0;      // dwords left out in all
  uint32_t kept_copies = 0;     // COPY_DATA→memory packets the compacted IB still has
  uint32_t copy_bytes = 0;      // bytes each copy writes (0: the copies differ in size)
  std::vector<uint64_t> dropped_dsts;
  std::string why;              // when !ok
};

// Compact `ib` (ndw dwords) into `out` as described above.
inline IbCompact compact_se_sections(const uint32_t* ib, uint32_t ndw, std::vector<uint32_t>& out) {
  IbCompact r;
  out.clear();
  out.reserve(ndw);
  std::vector<uint64_t> in_dsts;
  if (!ib_copy_dsts(ib, ndw, &in_dsts, &r.why)) return r;
  size_t pred_at = 0;       // index in `out` of the open PRED_EXEC's count dword (0 = none)
  uint32_t region_end = 0;  // its region's end in `ib`
  auto close_region = [&] {
    const uint32_t n = static_cast<uint32_t>(out.size() - (pred_at + 1));
    out[pred_at] = (out[pred_at] & ~kPredExecCountMask) | (n & kPredExecCountMask);
    pred_at = 0;
    region_end = 0;
  };
  for (uint32_t i = 0; i < ndw;) {
    if (region_end && i == region_end) close_region();
    const uint32_t h = ib[i];
    if (pm4_type(h) == 2) {  // filler
      out.push_back(h);
      ++i;
      continue;
    }
    const uint32_t len = pm4_len(h);
    bool se = false;
    if (pm4_gfx_index(ib + i, &se) && se) {
      // A per-SE section: only copies up to the next GRBM_GFX_INDEX write or region end?
      uint32_t j = i + len;
      uint32_t copies = 0;
      std::vector<uint64_t> dsts;
      while (j < ndw && !(region_end && j >= region_end)) {
        bool s2 = false;
        if (pm4_type(ib[j]) == 2) { ++j; continue; }
        if (pm4_gfx_index(ib + j, &s2)) break;
        if (!pm4_copy_to_mem(ib + j)) break;
        dsts.push_back(pm4_copy_dst(ib + j));
        ++copies;
        j += pm4_len(ib[j]);
      }
      bool s3 = false;
      const bool ends_clean = j >= ndw || (region_end && j == region_end) || pm4_gfx_index(ib + j, &s3);
      if (ends_clean && copies > 0) {
        r.dropped_copies += copies;
        r.dropped_dw += j - i;
        r.dropped_dsts.insert(r.dropped_dsts.end(), dsts.begin(), dsts.end());
        i = j;
        continue;
      }
    }
    if (pm4_op(h) == kPm4Nop) {  // a NOP left by the lean rewrite
      r.dropped_dw += len;
      i += len;
      continue;
    }
    const size_t at = out.size();
    out.insert(out.end(), ib + i, ib + i + len);
    if (pm4_op(h) == kPm4PredExec) {
      pred_at = at + 1;
      region_end = i + len + (ib[i + 1] & kPredExecCountMask);
    }
    i += len;
  }
  if (region_end) close_region();
  // Validate: the copy parses, and it writes exactly the kept results, in order.
  std::vector<uint64_t> out_dsts;
  if (!ib_copy_dsts(out.data(), static_cast<uint32_t>(out.size()), &out_dsts, &r.why)) {
    r.why = "compacted IB: " + r.why;
    return r;
  }
  std::vector<uint64_t> want;
  size_t d = 0;
  for (uint64_t x : in_dsts) {
    if (d < r.dropped_dsts.size() && r.dropped_dsts[d] == x) {
      ++d;
      continue;
    }
    want.push_back(x);
  }
  if (d != r.dropped_dsts.size() || want != out_dsts) {
    r.why = "compacted IB writes other results than the full one less the per-SE ones";
    return r;
  }
  if (r.dropped_copies == 0) {
    r.why = "no per-SE section";
    return r;
  }
  r.kept_copies = static_cast<uint32_t>(out_dsts.size());
  for (uint32_t i = 0; i < ndw;) {  // one copy size for every result copy, or 0
    if (pm4_type(ib[i]) == 2) { ++i; continue; }
    if (pm4_copy_to_mem(ib + i)) {
      const uint32_t b = pm4_copy_bytes(ib + i);
      if (r.copy_bytes == 0) r.copy_bytes = b;
      else if (r.copy_bytes != b) { r.copy_bytes = 0; break; }
    }
    i += pm4_len(ib[i]);
  }
  r.ok = true;
  return r;
}

}  // namespace kgs
