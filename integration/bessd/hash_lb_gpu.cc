// hash_lb_gpu.cc -- HashLB on MI355X: the bessd module `HashLB` replaced by a
// plugin of the same class name, gates, commands table (hash_lb.cc:75-79) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

class HashLB final : public GpuModule {
 public:
  static const gate_idx_t kNumOGates = MAX_GATES;  // hash_lb.h:45
  static const Commands cmds;

  CommandResponse Init(const bess::pb::HashLBArg &arg) {
    return CreateDeferred("HashLB", arg);
  }
  CommandResponse CommandSetMode(const bess::pb::HashLBCommandSetModeArg &arg) {
    return Run("set_mode", arg);
  }
  CommandResponse CommandSetGates(const bess::pb::HashLBCommandSetGatesArg &arg) {
    return Run("set_gates", arg);
  }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
  std::string GetDesc() const override { return Desc(); }
};

const Commands HashLB::cmds = {
    {"set_mode", "HashLBCommandSetModeArg", MODULE_CMD_FUNC(&HashLB::CommandSetMode),
     Command::THREAD_UNSAFE},
    {"set_gates", "HashLBCommandSetGatesArg", MODULE_CMD_FUNC(&HashLB::CommandSetGates),
     Command::THREAD_UNSAFE}};

ADD_MODULE(HashLB, "hash_lb", "splits packets on a flow basis with L2/L3/L4 header fields")
