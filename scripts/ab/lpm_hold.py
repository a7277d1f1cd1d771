# IPLookup (tbl16 in LDS, launch_line_wide): LPM_FORM selects
#   hold  line_kernel (a packet per lane, 1024 threads) holds H = LPM_HOLD
#         grid-stride results in registers and stores them together,
#         nontemporally, after their lookups (reading ops only);
#   slab  line_slab_kernel at one 512-thread workgroup per CU (tbl16 128 KB
#         + the 32 KB stage = 160 KB), whose reading ops already hold
#         kGateHold tiles.
import os
form = os.environ.get("LPM_FORM", "hold")
H = int(os.environ.get("LPM_HOLD", "8"))
if form == "hold":
    p = 'bess_amd/csrc/bg_line_dev.h'
    s = open(p).read()
    a = """  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < a.n;
       idx += step) {
    uint8_t *f"""
    b = """  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  constexpr int H = Op::kWrites ? 1 : %d;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < a.n;
       i0 += step * H) {
  uint16_t held[H];
#pragma unroll
  for (int hh = 0; hh < H; hh++) {
    const uint64_t idx = i0 + (uint64_t)hh * step;
    held[hh] = 0;
    if (idx >= a.n) break;
    uint8_t *f""" % H
    assert s.count(a) == 1
    s = s.replace(a, b)
    a = """    a.out[idx] = (uint16_t)Op::decide(a, lds, d, f);
    if constexpr (Op::kWrites) {
      uint4 *q = reinterpret_cast<uint4 *>(f);
#pragma unroll
      for (int c = Op::c0; c < Op::c1; c++)
        q[c] = make_uint4(d[4 * c], d[4 * c + 1], d[4 * c + 2], d[4 * c + 3]);
    }
  }
}"""
    b = """    held[hh] = (uint16_t)Op::decide(a, lds, d, f);
    if constexpr (Op::kWrites) {
      uint4 *q = reinterpret_cast<uint4 *>(f);
#pragma unroll
      for (int c = Op::c0; c < Op::c1; c++)
        q[c] = make_uint4(d[4 * c], d[4 * c + 1], d[4 * c + 2], d[4 * c + 3]);
    }
  }
#pragma unroll
  for (int hh = 0; hh < H; hh++) {
    const uint64_t idx = i0 + (uint64_t)hh * step;
    if (idx < a.n) __builtin_nontemporal_store(held[hh], a.out + idx);
  }
  }
}"""
    assert s.count(a) == 1
    s = s.replace(a, b)
    open(p, 'w').write(s)
elif form == "slab":
    p = 'bess_amd/csrc/bg_lpm.hip'
    s = open(p).read()
    a = """struct Lpm16LdsOp {  // (line_kernel only: launch_line_wide)
  using Args = LpmArgs;
  static constexpr bool kWrites = false;"""
    b = """struct Lpm16LdsOp {
  using Args = LpmArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 1;"""
    assert s.count(a) == 1
    s = s.replace(a, b)
    a = "  return launch_line_wide<Lpm16LdsOp>(a, num_cus, s);"
    assert s.count(a) == 1
    s = s.replace(a, "  return launch_line<Lpm16LdsOp>(a, num_cus, s);")
    open(p, 'w').write(s)
else:
    raise SystemExit("LPM_FORM: hold | slab")
