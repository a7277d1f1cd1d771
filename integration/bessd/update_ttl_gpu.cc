// update_ttl_gpu.cc -- UpdateTTL on MI355X: the bessd module `UpdateTTL` replaced by a
// plugin of the same class name, gates, commands table (none: update_ttl.h) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

class UpdateTTL final : public GpuModule {
 public:
  CommandResponse Init(const bess::pb::EmptyArg &arg) {
    return CreateDeferred("UpdateTTL", arg);
  }
  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
};

ADD_MODULE(UpdateTTL, "update_ttl", "decreases the IP TTL field by 1")
