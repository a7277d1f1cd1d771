// ip_checksum_gpu.cc -- IPChecksum on MI355X: the bessd module `IPChecksum` replaced by a
// plugin of the same class name, gates, commands table (none: ip_checksum.h) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

// The checksum is written into each frame in place (the staged header line
// goes back into the packet buffer before bg_module_process returns).
class IPChecksum final : public GpuModule {
 public:
  static const gate_idx_t kNumOGates = 2;  // ip_checksum.h:43

  CommandResponse Init(const bess::pb::IPChecksumArg &arg) {
    CommandResponse r = CreateDeferred("IPChecksum", arg);
    if (r.code() == 0) UsePacketPoolInPlace();  // frames in place, no staging copy
    return r;
  }
  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
};

ADD_MODULE(IPChecksum, "ip_checksum", "recomputes the IPv4 checksum")
