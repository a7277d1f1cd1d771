// update_ttl_module.cc -- UpdateTTL (core/modules/update_ttl.{h,cc}) with
// its ProcessBatch on the GPU (bg_update_ttl, bg_ttl.hip): no commands, no
// arguments; emits on gate 0 or drops.
#include <string.h>

#include <vector>

#include "../../include/bessgpu.h"
#include "module.h"

class UpdateTTL final : public Module {
 public:
  static const Commands kCmds;

  const Commands &cmds() const override { return kCmds; }

  CommandResponse Init(const bess::pb::EmptyArg &) { return CommandSuccess(); }

  int ProcessDevice(const bg_ctx &c, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    return bg_update_ttl(c.device, d_frames, stride, n, d_ogates, stream);
  }

  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    *lo = 0;
    *hi = 32;
    *writeback = true;
  }
};

const Commands UpdateTTL::kCmds = {};

ADD_MODULE_ARG(UpdateTTL, bess::pb::EmptyArg, "update_ttl",
               "decreases the IP TTL field by 1")
