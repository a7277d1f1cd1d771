// bg_ttl.hip -- gfx950 kernel for UpdateTTL::ProcessBatch
// (core/modules/update_ttl.cc:39-58): ttl > 1 -> ttl - 1 with the checksum
// updated incrementally (UpdateChecksum16(csum, 2, 1), checksum.h:520-560:
// fold(~csum + ~2 + 1), on the raw in-memory u16) and emit on gate 0;
// otherwise drop. The header line's chunks [0, C1) are read and written
// back whole (bg_line_dev.h writing op). Measured on MI355X (16M packets in
// 64 B slots): writing the whole 64-byte line (C1 = 4) takes 0.41 ms where
// writing bytes [0, 32) (C1 = 2) takes 0.62 ms -- a partial line costs the
// memory a read-modify-write. C1 = 2 remains for 32-byte staged windows
// (host pipe).
#include <hip/hip_runtime.h>
#include "bg_kernels.h"
#include "bg_launch.h"
#include "bg_line_dev.h"

namespace bg {
namespace {

template <int C1>
struct TtlOp {
  using Args = TtlArgs;
  static constexpr bool kWrites = true;
  static constexpr int kSlabPerCu = 2;
  static constexpr int c0 = 0, c1 = C1;
  static size_t lds_bytes(const TtlArgs &) { return 0; }
  __device__ static void stage(uint32_t *, const TtlArgs &) {}
  __device__ static uint32_t decide(const TtlArgs &, const uint32_t *,
                                    uint32_t (&d)[16], uint8_t *) {
    const uint32_t ttl = (d[5] >> 16) & 0xFF;  // byte 22
    if (ttl <= 1) return 8192;                 // DropPacket
    const uint32_t ck = d[6] & 0xFFFF;         // bytes 24..25, raw LE
    // UpdateChecksumWithIncrement(ck, ChecksumIncrement16(2, 1))
    uint32_t sum = (~ck & 0xFFFF) + ((~2u & 0xFFFF) + 1u);
    sum = (sum >> 16) + (sum & 0xFFFF);
    sum += sum >> 16;
    const uint32_t nck = ~sum & 0xFFFF;
    d[5] = (d[5] & 0xFF00FFFFu) | ((ttl - 1) << 16);
    d[6] = (d[6] & 0xFFFF0000u) | nck;
    return 0;
  }
};

}  // namespace

hipError_t launch_ttl(const TtlArgs &a, int num_cus, hipStream_t s) {
  if (a.stride >= 64) return launch_line<TtlOp<4>>(a, num_cus, s);
  return launch_line<TtlOp<2>>(a, num_cus, s);
}

}  // namespace bg
