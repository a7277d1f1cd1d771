// acl_gpu.cc -- ACL on MI355X: the bessd module `ACL` replaced by a
// plugin of the same class name, gates, commands table (acl.cc:36-40) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

// Passed packets leave on the gate they came in on, as in acl.cc:65-95.
class ACL final : public GpuModule {
 public:
  static const Commands cmds;

  CommandResponse Init(const bess::pb::ACLArg &arg) { return CreateDeferred("ACL", arg); }
  CommandResponse CommandAdd(const bess::pb::ACLArg &arg) { return Run("add", arg); }
  CommandResponse CommandClear(const bess::pb::EmptyArg &arg) { return Run("clear", arg); }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override { Forward(ctx, batch); }
};

const Commands ACL::cmds = {
    {"add", "ACLArg", MODULE_CMD_FUNC(&ACL::CommandAdd), Command::THREAD_UNSAFE},
    {"clear", "EmptyArg", MODULE_CMD_FUNC(&ACL::CommandClear), Command::THREAD_UNSAFE}};

ADD_MODULE(ACL, "acl", "ACL module from NetBricks")
