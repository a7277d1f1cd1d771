// wildcard_match_gpu.cc -- WildcardMatch on MI355X: the bessd module `WildcardMatch` replaced by a
// plugin of the same class name, gates, commands table (wildcard_match.cc:58-73) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

// A WildcardMatch ticket takes a ring workgroup ~20 us per 256 packets (its
// lookups' dependent L2 reads), so 512-packet slots, 8 in flight: the
// bounded-pool leg measured 512 x 8 against 1024 x 4 and 256 x 8 / x 16 on
// one box (profiles/r04_wm_plugin_slots.jsonl). (Compile-time: the
// harness's A/B builds set them.)
#ifndef BG_WM_PIPE_BATCH
#define BG_WM_PIPE_BATCH 512
#define BG_WM_PIPE_DEPTH 8
#endif

class WildcardMatch final : public GpuModule {
 public:
  static const gate_idx_t kNumOGates = MAX_GATES;  // wildcard_match.h:133
  static const Commands cmds;

  CommandResponse Init(const bess::pb::WildcardMatchArg &arg) {
    // served by a persistent ring on each device: small pipe slots
    return CreateDeferred("WildcardMatch", arg, BG_WM_PIPE_BATCH, BG_WM_PIPE_DEPTH);
  }
  CommandResponse GetInitialArg(const bess::pb::EmptyArg &arg) {
    bess::pb::WildcardMatchArg r;
    return Run("get_initial_arg", arg, &r);
  }
  CommandResponse GetRuntimeConfig(const bess::pb::EmptyArg &arg) {
    bess::pb::WildcardMatchConfig r;
    return Run("get_runtime_config", arg, &r);
  }
  CommandResponse SetRuntimeConfig(const bess::pb::WildcardMatchConfig &arg) {
    return Run("set_runtime_config", arg);
  }
  CommandResponse CommandAdd(const bess::pb::WildcardMatchCommandAddArg &arg) {
    return Run("add", arg);
  }
  CommandResponse CommandDelete(const bess::pb::WildcardMatchCommandDeleteArg &arg) {
    return Run("delete", arg);
  }
  CommandResponse CommandClear(const bess::pb::EmptyArg &arg) { return Run("clear", arg); }
  CommandResponse CommandSetDefaultGate(
      const bess::pb::WildcardMatchCommandSetDefaultGateArg &arg) {
    return Run("set_default_gate", arg);
  }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
  std::string GetDesc() const override { return Desc(); }
};

const Commands WildcardMatch::cmds = {
    {"get_initial_arg", "EmptyArg", MODULE_CMD_FUNC(&WildcardMatch::GetInitialArg),
     Command::THREAD_SAFE},
    {"get_runtime_config", "EmptyArg", MODULE_CMD_FUNC(&WildcardMatch::GetRuntimeConfig),
     Command::THREAD_SAFE},
    {"set_runtime_config", "WildcardMatchConfig",
     MODULE_CMD_FUNC(&WildcardMatch::SetRuntimeConfig), Command::THREAD_UNSAFE},
    {"add", "WildcardMatchCommandAddArg", MODULE_CMD_FUNC(&WildcardMatch::CommandAdd),
     Command::THREAD_UNSAFE},
    {"delete", "WildcardMatchCommandDeleteArg",
     MODULE_CMD_FUNC(&WildcardMatch::CommandDelete), Command::THREAD_UNSAFE},
    {"clear", "EmptyArg", MODULE_CMD_FUNC(&WildcardMatch::CommandClear),
     Command::THREAD_UNSAFE},
    {"set_default_gate", "WildcardMatchCommandSetDefaultGateArg",
     MODULE_CMD_FUNC(&WildcardMatch::CommandSetDefaultGate), Command::THREAD_SAFE}};

ADD_MODULE(WildcardMatch, "wm", "Multi-field classifier with a wildcard match table")
