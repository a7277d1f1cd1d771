// bg_launch.h -- host-side launch policy shared by the kernel launchers.
//
// The product library (libbessgpu.so) reads no environment on its launch
// path: every launch shape is a measured constant. Two things vary:
//
//   * path_flags(): bg_set_path_flags() picks among kernels that compute the
//     SAME result (table in LDS or L2, coalesced slab or lane-per-packet,
//     WildcardMatch tag words or key filter), so the parity tests can run
//     every path against the oracle. One relaxed atomic load per launch.
//   * knob(): A/B measurement knobs (scripts/variants.py). In the product
//     build knob(name, dflt) is the constant dflt; only the separate
//     measurement build libbessgpu_ab.so (-DBG_AB, `make ab`) reads BG_*
//     environment variables, and only that build compiles the A/B-only
//     kernel variants.
//
// occupancy() memoises hipOccupancyMaxActiveBlocksPerMultiprocessor per
// (kernel, block, LDS bytes) in a lock-free list: launches from many worker
// threads never serialise on it.
#ifndef BESS_AMD_BG_LAUNCH_H_
#define BESS_AMD_BG_LAUNCH_H_

#include <stddef.h>
#include <stdint.h>

namespace bg {

constexpr uint32_t kPathForceLds = 1;   // stage tables in LDS even for small launches
constexpr uint32_t kPathNoLds = 2;      // probe tables in L2 (never LDS)
constexpr uint32_t kPathNoSlab = 4;     // lane-per-packet kernels, never the slab shape
constexpr uint32_t kPathWmNoTags = 8;   // WildcardMatch: key filter, not tag words
constexpr uint32_t kPathAclScan = 16;   // ACL: the rule scan with scalar rule loads
constexpr uint32_t kPathAclBv = 32;     // ACL: per-dimension bit vectors
constexpr uint32_t kPathAclLds = 64;    // ACL: the rule scan from LDS (not the tree)
constexpr uint32_t kPathLpmDir24 = 128;  // IPLookup: DIR-24-8 (not DIR-16-8-8)
constexpr uint32_t kPathPipeNoRing = 256;  // pipes launch per slot (no ring)
constexpr uint32_t kPathWmNoJit = 512;   // WildcardMatch: never the run-time compiled kernel
constexpr uint32_t kPathRingHostDesc = 1024;  // rings: descriptors in pinned host memory
constexpr uint32_t kPathWmStream = 2048;  // WildcardMatch: the streamed tag-word form
constexpr uint32_t kPathAll = 4095;

uint32_t path_flags();

#ifdef BG_AB
int knob(const char *name, int dflt);
#else
constexpr int knob(const char *, int dflt) { return dflt; }
#endif

int occupancy(const void *kernel, int block, size_t lds, int dflt);

// the WildcardMatch streamed form's ring slots (wm_stream_slots; the A/B
// build caps them with BG_WM_STREAM_SLOTS, which also picks the shallower
// producer depth)
uint32_t stream_slots(uint32_t nbp, uint32_t kw);

// the WildcardMatch tag-word kernels' line form applies (dense 64 B slots,
// 16 B-aligned slab, the window two chunks inside the slot, its LDS fits)
// -- measured slower than the pair loads (C4 slab 0.1661 against 0.1532
// ms), so only the A/B build selects it (BG_WM_LINE=1)
struct WmArgs;
bool wm_line_ok(const WmArgs &a);

}  // namespace bg

#endif  // BESS_AMD_BG_LAUNCH_H_
