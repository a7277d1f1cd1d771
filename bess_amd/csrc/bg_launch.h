// bg_launch.h -- host-side launch policy shared by the kernel launchers.
//
// The library reads no environment: every launch shape is a measured
// constant (the variants they were measured against, rounds 1-5, are in
// DESIGN §3 and profiles/). One thing varies: path_flags() --
// bg_set_path_flags() picks among kernels that compute the SAME result
// (table in LDS or L2, coalesced slab or lane-per-packet, WildcardMatch tag
// words or key filter), so the parity tests can run every path against the
// oracle. One relaxed atomic load per launch.
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
constexpr uint32_t kPathAll = 2047;

uint32_t path_flags();

int occupancy(const void *kernel, int block, size_t lds, int dflt);

}  // namespace bg

#endif  // BESS_AMD_BG_LAUNCH_H_
