// rewrite_gpu.cc -- Rewrite on MI355X: the bessd module `Rewrite` replaced by a
// plugin of the same class name, gates, commands table (rewrite.cc:7-12) and Init
// argument, forwarding to libbessgpu.so (bg_rewrite_*).
#include "gpu_module.h"

// Each packet's data becomes the next template, round robin across
// batches (rewrite.cc:72-113): the packets' buffers are written from the
// GPU through the calling worker's staging, data_off = SNBUF_HEADROOM and
// both lengths = the template's size; the batch goes on to gate 0.
class Rewrite final : public GpuModule {
 public:
  static const Commands cmds;

  ~Rewrite() {
    if (rw_) bg_rewrite_destroy(rw_);
  }

  CommandResponse Init(const bess::pb::RewriteArg &arg) {
    if (bg_rewrite_create(&rw_) < 0) return CommandFailure(ENOMEM, "%s", bg_last_error());
    return CommandAdd(arg);
  }
  CommandResponse CommandAdd(const bess::pb::RewriteArg &arg) {
    const std::string b = arg.SerializeAsString();
    const int r = bg_rewrite_add_pb(rw_, b.data(), b.size());
    if (r < 0) return CommandFailure(-r, "%s", bg_last_error());
    return CommandSuccess();
  }
  CommandResponse CommandClear(const bess::pb::EmptyArg &) {
    bg_rewrite_clear(rw_);
    return CommandSuccess();
  }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override {
    const int n = batch->cnt();
    uint8_t *bufs[bess::PacketBatch::kMaxBurst] = {};
    uint16_t head[bess::PacketBatch::kMaxBurst] = {};
    uint32_t len[bess::PacketBatch::kMaxBurst] = {};
    for (int i = 0; i < n; i++)  // the mbuf's buffer: headroom, then data
      bufs[i] = reinterpret_cast<uint8_t *>(batch->pkts()[i]) + SNBUF_HEADROOM_OFF;
    if (bg_rewrite_count(rw_) > 0) {
      if (bg_rewrite_process_host(rw_, 0, bufs, SNBUF_HEADROOM + SNBUF_DATA, (size_t)n,
                                  SNBUF_HEADROOM, head, len, nullptr) < 0) {
        for (int i = 0; i < n; i++) DropPacket(ctx, batch->pkts()[i]);
        return;
      }
      for (int i = 0; i < n; i++) {
        bess::Packet *pkt = batch->pkts()[i];
        pkt->set_data_off(head[i]);
        pkt->set_total_len(len[i]);
        pkt->set_data_len((uint16_t)len[i]);
      }
    }
    RunNextModule(ctx, batch);
  }

 private:
  bg_rewrite *rw_ = nullptr;
};

const Commands Rewrite::cmds = {
    {"add", "RewriteArg", MODULE_CMD_FUNC(&Rewrite::CommandAdd), Command::THREAD_UNSAFE},
    {"clear", "EmptyArg", MODULE_CMD_FUNC(&Rewrite::CommandClear), Command::THREAD_UNSAFE}};

ADD_MODULE(Rewrite, "rewrite", "replaces entire packet data")
