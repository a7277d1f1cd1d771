// nat_gpu.cc -- NAT (dynamic) on MI355X: the bessd module `NAT` replaced by a
// plugin of the same class name, gates, commands table (nat.cc:56-62) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

// Input gate 0 maps internal sources (creating mappings) and emits on 1,
// input gate 1 maps external destinations and emits on 0; the mapping
// clock is ctx->current_ns (nat.cc:321-363); both go over with each batch.
class NAT final : public GpuModule {
 public:
  NAT() { max_allowed_workers_ = 1; }  // Module's default (nat.h sets none)

  static const gate_idx_t kNumIGates = 2;  // nat.h:141-142
  static const gate_idx_t kNumOGates = 2;
  static const Commands cmds;

  CommandResponse Init(const bess::pb::NATArg &arg) { return Create("NAT", arg); }
  CommandResponse GetInitialArg(const bess::pb::EmptyArg &arg) {
    bess::pb::NATArg r;
    return Run("get_initial_arg", arg, &r);
  }
  CommandResponse GetRuntimeConfig(const bess::pb::EmptyArg &arg) {
    return Run("get_runtime_config", arg);
  }
  CommandResponse SetRuntimeConfig(const bess::pb::EmptyArg &arg) {
    return Run("set_runtime_config", arg);
  }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
  std::string GetDesc() const override { return Desc(); }
};

const Commands NAT::cmds = {
    {"get_initial_arg", "EmptyArg", MODULE_CMD_FUNC(&NAT::GetInitialArg),
     Command::THREAD_SAFE},
    {"get_runtime_config", "EmptyArg", MODULE_CMD_FUNC(&NAT::GetRuntimeConfig),
     Command::THREAD_SAFE},
    {"set_runtime_config", "EmptyArg", MODULE_CMD_FUNC(&NAT::SetRuntimeConfig),
     Command::THREAD_SAFE}};

ADD_MODULE(NAT, "nat", "Dynamic Network address/port translator")
