# line_slab_kernel (reading ops): results held in LDS instead of registers,
# as em_slab_kernel does beside an LDS table: up to LH_MAX tiles per wave,
# what the CU's LDS (split over the op's kSlabPerCu workgroups) leaves after
# the op's tables and the stages; the tile loop is not unrolled; the held
# results leave 16 B per lane. LH_MAX from the environment (128).
import os
HMAX = int(os.environ.get("LH_MAX", "128"))
p = 'bess_amd/csrc/bg_line_dev.h'
s = open(p).read()

a = """template <class Op>
__global__ __launch_bounds__(kLineBlock) void line_slab_kernel(typename Op::Args a,
                                                              uint32_t stage_words) {"""
b = """template <class Op>
__host__ __device__ constexpr uint32_t line_hold_tiles(uint32_t tab_bytes) {
  if (Op::kWrites) return 0u;
  const uint32_t budget = kLdsPerCu / Op::kSlabPerCu;
  const uint32_t stage = (kLineBlock / 64) * 4096u, per_tile = (kLineBlock / 64) * 128u;
  const uint32_t room = tab_bytes + stage < budget ? budget - tab_bytes - stage : 0u;
  const uint32_t h = (room / per_tile) & ~7u;
  return h < %du ? h : %du;
}

template <class Op>
__global__ __launch_bounds__(kLineBlock) void line_slab_kernel(typename Op::Args a,
                                                              uint32_t stage_words) {""" % (HMAX, HMAX)
assert s.count(a) == 1
s = s.replace(a, b)

a = """  constexpr int H = Op::kWrites ? 1 : kGateHold;
  if (t < ntiles) load_tile(t);"""
b = """  const uint32_t hl = line_hold_tiles<Op>(stage_words * 4);
  if (t < ntiles) load_tile(t);
  if (hl) {
    uint16_t *hold = reinterpret_cast<uint16_t *>(lds + stage_words + kWaves * 1024) +
                     (size_t)wid * hl * 64;
    const bool al16 = ((uintptr_t)a.out & 15) == 0;
    for (uint64_t t0 = t; t0 < ntiles; t0 += nwaves * hl) {
#pragma unroll 1
      for (uint32_t h = 0; h < hl; h++) {
        const uint64_t tt = t0 + (uint64_t)h * nwaves;
        if (tt >= ntiles) break;
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const uint32_t u = c * 64 + lane;
          stage[line_stage_unit(u >> 2, u & 3)] = v[c];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (tt + nwaves < ntiles) load_tile(tt + nwaves);
        uint32_t d[16];
#pragma unroll
        for (int c = 0; c < 4; c++) {
          uint4 x = make_uint4(0, 0, 0, 0);
          if (c >= Op::c0 && c < Op::c1) x = stage[line_stage_unit(lane, c)];
          d[4 * c] = x.x;
          d[4 * c + 1] = x.y;
          d[4 * c + 2] = x.z;
          d[4 * c + 3] = x.w;
        }
        const uint64_t idx = tt * 64 + lane;
        uint16_t g = 0;
        if (idx < a.n) {
          uint8_t *f = const_cast<uint8_t *>(a.frames) + idx * 64;
          g = (uint16_t)Op::decide(a, lds, d, f);
        }
        hold[h * 64 + lane] = g;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
#pragma unroll 1
      for (uint32_t i = 0; i < hl; i += 8) {
        const uint32_t h = i + (lane >> 3);
        const uint64_t idx = (t0 + (uint64_t)h * nwaves) * 64 + (lane & 7) * 8;
        if (idx >= a.n) continue;
        const uint4 x = reinterpret_cast<const uint4 *>(hold + h * 64)[lane & 7];
        if (al16 && idx + 8 <= a.n) {
          st_stream(reinterpret_cast<uint4 *>(a.out + idx), x);
        } else {
          const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
          for (int j = 0; j < 8 && idx + j < a.n; j++)
            a.out[idx + j] = (uint16_t)(xs[j >> 1] >> (16 * (j & 1)));
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return;
  }
  constexpr int H = Op::kWrites ? 1 : kGateHold;"""
assert s.count(a) == 1
s = s.replace(a, b)

a = """    auto kern = line_slab_kernel<Op>;
    const size_t lds = tab + (size_t)(kLineBlock / 64) * 4096;"""
b = """    auto kern = line_slab_kernel<Op>;
    const size_t lds = tab + (size_t)(kLineBlock / 64) * 4096 +
                       (size_t)line_hold_tiles<Op>((uint32_t)tab) * (kLineBlock / 64) * 128;"""
assert s.count(a) == 1
s = s.replace(a, b)
open(p, 'w').write(s)
