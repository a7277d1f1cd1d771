// exact_match_gpu.cc -- ExactMatch on MI355X: the bessd module `ExactMatch` replaced by a
// plugin of the same class name, gates, commands table (exact_match.cc:45-60) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

class ExactMatch final : public GpuModule {
 public:
  static const gate_idx_t kNumOGates = MAX_GATES;  // exact_match.h:50
  static const Commands cmds;

  CommandResponse Init(const bess::pb::ExactMatchArg &arg) {
    // served by a persistent ring on each device: small pipe slots
    return CreateDeferred("ExactMatch", arg, kRingPipeBatch, kRingPipeDepth);
  }
  CommandResponse GetInitialArg(const bess::pb::EmptyArg &arg) {
    bess::pb::ExactMatchArg r;
    return Run("get_initial_arg", arg, &r);
  }
  CommandResponse GetRuntimeConfig(const bess::pb::EmptyArg &arg) {
    bess::pb::ExactMatchConfig r;
    return Run("get_runtime_config", arg, &r);
  }
  CommandResponse SetRuntimeConfig(const bess::pb::ExactMatchConfig &arg) {
    return Run("set_runtime_config", arg);
  }
  CommandResponse CommandAdd(const bess::pb::ExactMatchCommandAddArg &arg) {
    return Run("add", arg);
  }
  CommandResponse CommandDelete(const bess::pb::ExactMatchCommandDeleteArg &arg) {
    return Run("delete", arg);
  }
  CommandResponse CommandClear(const bess::pb::EmptyArg &arg) { return Run("clear", arg); }
  CommandResponse CommandSetDefaultGate(
      const bess::pb::ExactMatchCommandSetDefaultGateArg &arg) {
    return Run("set_default_gate", arg);
  }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
  std::string GetDesc() const override { return Desc(); }
};

const Commands ExactMatch::cmds = {
    {"get_initial_arg", "EmptyArg", MODULE_CMD_FUNC(&ExactMatch::GetInitialArg),
     Command::THREAD_SAFE},
    {"get_runtime_config", "EmptyArg", MODULE_CMD_FUNC(&ExactMatch::GetRuntimeConfig),
     Command::THREAD_SAFE},
    {"set_runtime_config", "ExactMatchConfig",
     MODULE_CMD_FUNC(&ExactMatch::SetRuntimeConfig), Command::THREAD_UNSAFE},
    {"add", "ExactMatchCommandAddArg", MODULE_CMD_FUNC(&ExactMatch::CommandAdd),
     Command::THREAD_UNSAFE},
    {"delete", "ExactMatchCommandDeleteArg", MODULE_CMD_FUNC(&ExactMatch::CommandDelete),
     Command::THREAD_UNSAFE},
    {"clear", "EmptyArg", MODULE_CMD_FUNC(&ExactMatch::CommandClear), Command::THREAD_UNSAFE},
    {"set_default_gate", "ExactMatchCommandSetDefaultGateArg",
     MODULE_CMD_FUNC(&ExactMatch::CommandSetDefaultGate), Command::THREAD_SAFE}};

ADD_MODULE(ExactMatch, "em", "Multi-field classifier with an exact match table")
