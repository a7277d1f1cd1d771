// bg_launch.cc -- launch policy (bg_launch.h) and bg_set_path_flags.
#include "bg_launch.h"

#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <atomic>

#include "../../include/bessgpu.h"
#include "bg_internal.h"
#include "bg_kernels.h"

namespace bg {

namespace {
std::atomic<uint32_t> g_path{0};

struct OccEnt {
  const void *kernel;
  size_t lds;
  int block, occ;
  OccEnt *next;
};
std::atomic<OccEnt *> g_occ{nullptr};
}  // namespace

#ifdef BG_AB
int knob(const char *name, int dflt) {
  const char *v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}
#endif

uint32_t path_flags() {
  uint32_t f = g_path.load(std::memory_order_relaxed);
#ifdef BG_AB  // scripts/variants.py selects paths through the environment
  if (knob("BG_FORCE_LDS", 0)) f |= kPathForceLds;
  if (knob("BG_NOLDS", 0)) f |= kPathNoLds;
  if (knob("BG_NO_SLAB", 0)) f |= kPathNoSlab;
  if (knob("BG_WM_STREAM", 0)) f |= kPathWmStream;
#endif
  return f;
}

// Entries are pushed once and never removed, so readers walk the list
// without a lock; two threads racing on a new key both compute the same
// answer and at worst push it twice.
uint32_t stream_slots(uint32_t nbp, uint32_t kw) {
  uint32_t r = wm_stream_slots(nbp, kw);
#ifdef BG_AB
  const int cap = knob("BG_WM_STREAM_SLOTS", 0);
  if (cap > 0 && r > (uint32_t)cap)
    r = cap > kStreamProducers * kStreamDepth + 4 ? (uint32_t)cap : 0u;
#endif
  return r;
}

bool wm_line_ok(const WmArgs &a) {
  return a.stride == 64 && (reinterpret_cast<uintptr_t>(a.frames) & 15) == 0 &&
         a.fp.win_lo % 16 == 0 && a.fp.win_lo + 32 <= 64 &&
         wm_line_lds_bytes(a.t.nbp, a.t.kw) <= kLdsMax && knob("BG_WM_LINE", 0) != 0;
}

int occupancy(const void *kernel, int block, size_t lds, int dflt) {
  for (OccEnt *e = g_occ.load(std::memory_order_acquire); e; e = e->next)
    if (e->kernel == kernel && e->lds == lds && e->block == block) return e->occ;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, block, lds) !=
          hipSuccess ||
      occ <= 0)
    occ = dflt;
  OccEnt *n = new OccEnt{kernel, lds, block, occ, nullptr};
  n->next = g_occ.load(std::memory_order_relaxed);
  while (!g_occ.compare_exchange_weak(n->next, n, std::memory_order_release,
                                      std::memory_order_relaxed)) {
  }
  return occ;
}

}  // namespace bg

extern "C" int bg_set_path_flags(uint32_t flags) {
  if (flags & ~bg::kPathAll) return bg::fail(EINVAL, "unknown path flags 0x%x", flags);
  if ((flags & bg::kPathForceLds) && (flags & bg::kPathNoLds))
    return bg::fail(EINVAL, "BG_PATH_FORCE_LDS and BG_PATH_NO_LDS exclude each other");
  bg::g_path.store(flags, std::memory_order_relaxed);
  return 0;
}

extern "C" uint32_t bg_get_path_flags(void) { return bg::path_flags(); }

extern "C" int bg_is_ab_build(void) {
#ifdef BG_AB
  return 1;
#else
  return 0;
#endif
}
