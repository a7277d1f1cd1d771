// static_nat_gpu.cc -- StaticNAT on MI355X: the bessd module `StaticNAT` replaced by a
// plugin of the same class name, gates, commands table (static_nat.cc:38-44) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

// Input gate 0 translates sources and emits on 1, input gate 1 translates
// destinations and emits on 0 (static_nat.cc:179-187).
class StaticNAT final : public GpuModule {
 public:
  StaticNAT() { max_allowed_workers_ = 1; }  // Module's default (static_nat.h)

  static const gate_idx_t kNumIGates = 2;  // static_nat.h:51-52
  static const gate_idx_t kNumOGates = 2;
  static const Commands cmds;

  CommandResponse Init(const bess::pb::StaticNATArg &arg) {
    return CreateDeferred("StaticNAT", arg);
  }
  CommandResponse GetInitialArg(const bess::pb::EmptyArg &arg) {
    bess::pb::StaticNATArg r;
    return Run("get_initial_arg", arg, &r);
  }
  CommandResponse GetRuntimeConfig(const bess::pb::EmptyArg &arg) {
    return Run("get_runtime_config", arg);
  }
  CommandResponse SetRuntimeConfig(const bess::pb::EmptyArg &arg) {
    return Run("set_runtime_config", arg);
  }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
};

const Commands StaticNAT::cmds = {
    {"get_initial_arg", "EmptyArg", MODULE_CMD_FUNC(&StaticNAT::GetInitialArg),
     Command::THREAD_SAFE},
    {"get_runtime_config", "EmptyArg", MODULE_CMD_FUNC(&StaticNAT::GetRuntimeConfig),
     Command::THREAD_SAFE},
    {"set_runtime_config", "EmptyArg", MODULE_CMD_FUNC(&StaticNAT::SetRuntimeConfig),
     Command::THREAD_SAFE}};

ADD_MODULE(StaticNAT, "static_nat", "Static network address translator")
