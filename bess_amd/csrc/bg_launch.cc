// bg_launch.cc -- launch policy (bg_launch.h) and bg_set_path_flags.
#include "bg_launch.h"

#include <errno.h>
#include <hip/hip_runtime.h>

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

uint32_t path_flags() { return g_path.load(std::memory_order_relaxed); }

// Entries are pushed once and never removed, so readers walk the list
// without a lock; two threads racing on a new key both compute the same
// answer and at worst push it twice.
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
