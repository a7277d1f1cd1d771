// l4_checksum_gpu.cc -- L4Checksum on MI355X: the bessd module `L4Checksum` replaced by a
// plugin of the same class name, gates, commands table (none: l4_checksum.h) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

class L4Checksum final : public GpuModule {
 public:
  static const gate_idx_t kNumOGates = 2;          // l4_checksum.h:42
  static const gate_idx_t kNumIGates = MAX_GATES;  // l4_checksum.h:43

  CommandResponse Init(const bess::pb::L4ChecksumArg &arg) {
    CommandResponse r = CreateDeferred("L4Checksum", arg);
    if (r.code() == 0) UsePacketPoolInPlace();  // frames in place, no staging copy
    return r;
  }
  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
};

ADD_MODULE(L4Checksum, "l4_checksum", "recomputes the TCP/Ipv4 and UDP/IPv4 checksum")
