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

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override {
    ProcessPackets(ctx, batch->pkts(), (size_t)batch->cnt());
  }

  // synchronous host path: bytes [0, 32) round-trip through the device
  int ProcessPackets(Context *ctx, bess::Packet *const *pkts,
                     size_t cnt) override {
    if (cnt == 0) return 0;
    const size_t w = 32;
    std::vector<uint8_t> h(cnt * w);
    for (size_t i = 0; i < cnt; i++)
      memcpy(h.data() + i * w, pkts[i]->head_data<uint8_t *>(), w);
    void *d_in = nullptr, *d_out = nullptr;
    int rc = bg_malloc(device_, h.size(), &d_in);
    if (rc == 0) rc = bg_malloc(device_, cnt * 2, &d_out);
    if (rc == 0) rc = bg_memcpy_h2d(d_in, h.data(), h.size(), nullptr);
    if (rc == 0)
      rc = bg_update_ttl(device_, d_in, w, cnt, static_cast<uint16_t *>(d_out),
                         nullptr);
    std::vector<uint16_t> g(cnt);
    if (rc == 0) rc = bg_memcpy_d2h(g.data(), d_out, cnt * 2, nullptr);
    if (rc == 0) rc = bg_memcpy_d2h(h.data(), d_in, h.size(), nullptr);
    if (rc == 0) rc = bg_stream_sync(nullptr);
    if (d_in) bg_free(d_in);
    if (d_out) bg_free(d_out);
    if (rc < 0) {
      for (size_t i = 0; i < cnt; i++) DropPacket(ctx, pkts[i]);
      return rc;
    }
    for (size_t i = 0; i < cnt; i++) {
      if (g[i] == DROP_GATE) {
        DropPacket(ctx, pkts[i]);
      } else {
        memcpy(pkts[i]->head_data<uint8_t *>(), h.data() + i * w, w);
        EmitPacket(ctx, pkts[i], 0);
      }
    }
    return 0;
  }

  int ProcessDevice(void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    return bg_update_ttl(device_, d_frames, stride, n, d_ogates, stream);
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
