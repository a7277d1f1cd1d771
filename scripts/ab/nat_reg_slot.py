# NAT's slab kernel with a tile-uniform register path (measured slower in
# r06al: 0.5092-0.5115 against 0.4970-0.4977 ms per 16 M packets, not kept):
# when every live lane's packet has IHL 5, the lane's 64-byte slot is read
# from the LDS stage into 16 registers, looked up and stamped there through
# RegSlot5 (every offset a constant but the direction-dependent ones, which
# select over the 16 words), and written back to the stage.
p = "bess_amd/csrc/bg_dnat.hip"
s = open(p).read()
R = [("""  __device__ uint32_t u8(uint32_t o) const { return o < lim ? p[o] : 0u; }""",
      """  __device__ uint32_t l4() const { return 14 + ((u8(14) & 0x0Fu) << 2); }
  __device__ uint32_t u8(uint32_t o) const { return o < lim ? p[o] : 0u; }"""),
     ("""  __device__ uint32_t u8(uint32_t o) const { return o < 64 ? stage[at(o)] : 0u; }""",
      """  __device__ uint32_t l4() const { return 14 + ((u8(14) & 0x0Fu) << 2); }
  __device__ uint32_t u8(uint32_t o) const { return o < 64 ? stage[at(o)] : 0u; }"""),
     ("""// fold(~ck + incr) (UpdateChecksumWithIncrement, checksum.h:535-538)""",
      """struct RegSlot5 {
  uint32_t (&d)[16];
  __device__ uint32_t l4() const { return 34; }
  __device__ uint32_t word(uint32_t k) const {
    uint32_t w = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) w = k == j ? d[j] : w;
    return w;
  }
  __device__ uint32_t u8(uint32_t o) const { return (word(o >> 2) >> ((o & 3) * 8)) & 0xFFu; }
  __device__ uint32_t u16(uint32_t o) const { return (word(o >> 2) >> ((o & 2) * 8)) & 0xFFFFu; }
  __device__ void put16(uint32_t o, uint32_t v) const {
    const uint32_t sh = (o & 2) * 8, m = ~(0xFFFFu << sh), x = (v & 0xFFFFu) << sh;
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) d[j] = (o >> 2) == j ? (d[j] & m) | x : d[j];
  }
};

// fold(~ck + incr) (UpdateChecksumWithIncrement, checksum.h:535-538)"""),
     ("""__device__ __forceinline__ uint64_t endpoint(const F &f, uint32_t dir) {
  const uint32_t l4 = 14 + ((f.u8(14) & 0x0Fu) << 2);""",
      """__device__ __forceinline__ uint64_t endpoint(const F &f, uint32_t dir) {
  const uint32_t l4 = f.l4();"""),
     ("""                                      uint32_t dir) {
  const uint32_t l4 = 14 + ((f.u8(14) & 0x0Fu) << 2);""",
      """                                      uint32_t dir) {
  const uint32_t l4 = f.l4();"""),
     ("""    const uint64_t idx = t * 64 + lane;
    fused_one(a, me, idx, idx < a.n);
    lds_fence();""",
      """    const uint64_t idx = t * 64 + lane;
    const bool live = idx < a.n;
    if (__all(!live || (me.u8(14) & 0x0Fu) == 5u)) {
      uint32_t d[16];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const uint4 x = stage[lane * 4 + ((c + (lane >> 2)) & 3)];
        d[4 * c] = x.x;
        d[4 * c + 1] = x.y;
        d[4 * c + 2] = x.z;
        d[4 * c + 3] = x.w;
      }
      fused_one(a, RegSlot5{d}, idx, live);
#pragma unroll
      for (int c = 0; c < 4; c++)
        stage[lane * 4 + ((c + (lane >> 2)) & 3)] =
            make_uint4(d[4 * c], d[4 * c + 1], d[4 * c + 2], d[4 * c + 3]);
    } else {
      fused_one(a, me, idx, live);
    }
    lds_fence();""")]
for a, b in R:
    assert s.count(a) == 1, a[:50]
    s = s.replace(a, b)
open(p, "w").write(s)
