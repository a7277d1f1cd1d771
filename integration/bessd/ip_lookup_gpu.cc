// ip_lookup_gpu.cc -- IPLookup on MI355X: the bessd module `IPLookup` replaced by a
// plugin of the same class name, gates, commands table (ip_lookup.cc:48-54) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

class IPLookup final : public GpuModule {
 public:
  static const gate_idx_t kNumOGates = MAX_GATES;  // ip_lookup.h:43
  static const Commands cmds;

  CommandResponse Init(const bess::pb::IPLookupArg &arg) {
    return CreateDeferred("IPLookup", arg);
  }
  CommandResponse CommandAdd(const bess::pb::IPLookupCommandAddArg &arg) {
    return Run("add", arg);
  }
  CommandResponse CommandDelete(const bess::pb::IPLookupCommandDeleteArg &arg) {
    return Run("delete", arg);
  }
  CommandResponse CommandClear(const bess::pb::EmptyArg &arg) { return Run("clear", arg); }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
};

const Commands IPLookup::cmds = {
    {"add", "IPLookupCommandAddArg", MODULE_CMD_FUNC(&IPLookup::CommandAdd),
     Command::THREAD_UNSAFE},
    {"delete", "IPLookupCommandDeleteArg", MODULE_CMD_FUNC(&IPLookup::CommandDelete),
     Command::THREAD_UNSAFE},
    {"clear", "EmptyArg", MODULE_CMD_FUNC(&IPLookup::CommandClear), Command::THREAD_UNSAFE}};

ADD_MODULE(IPLookup, "ip_lookup", "performs Longest Prefix Match on IPv4 packets")
