// gpu_module.h -- the part every libbessgpu.so-backed bessd module shares.
//
// Drop these files into bessd's core/modules/ (they include "../module.h"
// and "../pb/module_msg.pb.h" like the built-in modules) and link the
// plugin with -lbessgpu. Each *_gpu.cc declares the same class name,
// gates, commands table and Init argument as the module it replaces, and
// forwards everything to the C ABI (include/bessgpu.h):
//   Init                  -> bg_module_create(<class>, <Class>Arg bytes)
//   a command             -> bg_module_command(name, arg bytes) (+ response)
//   ProcessBatch          -> bg_module_process (heads in, a gate per packet)
//   GetDesc               -> bg_module_desc
// and maps the gates back onto bessd's EmitPacket / DropPacket, whose own
// check drops a packet sent to an out-of-range or unconnected gate
// (core/module.h:546-549).
#ifndef BESS_MODULES_GPU_MODULE_H_
#define BESS_MODULES_GPU_MODULE_H_

#include <string>

#include "../module.h"
#include "../pb/module_msg.pb.h"
#include "bessgpu.h"

class GpuModule : public Module {
 public:
  void DeInit() override {
    bg_module_destroy(m_);
    m_ = nullptr;
  }

 protected:
  CommandResponse Create(const char *mclass, const google::protobuf::Message &arg) {
    const std::string b = arg.SerializeAsString();
    const int rc = bg_module_create(mclass, b.data(), b.size(), &m_);
    return rc < 0 ? CommandFailure(-rc, "%s", bg_last_error()) : CommandSuccess();
  }

  // `cmd` with its argument; the C side checks it and answers with the
  // reference's errno and message. resp: the command's response message.
  CommandResponse Run(const char *cmd, const google::protobuf::Message &arg,
                      google::protobuf::Message *resp = nullptr) {
    const std::string in = arg.SerializeAsString();
    std::string out(1 << 16, '\0');
    size_t len = out.size();
    int rc = bg_module_command(m_, cmd, in.data(), in.size(), &out[0], &len);
    if (rc == -ENOBUFS && len > out.size()) {  // a larger response (get_*): again
      out.resize(len);
      rc = bg_module_command(m_, cmd, in.data(), in.size(), &out[0], &len);
    }
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    if (!resp) return CommandSuccess();
    resp->ParseFromArray(out.data(), (int)len);
    return CommandSuccess(*resp);
  }

  // bessd's per-call Context as the C ABI's bg_ctx: ctx->current_igate
  // (ACL, StaticNAT, NAT act on it) and ctx->current_ns (NAT's clock) go
  // with the call, never into the shared module
  static bg_ctx CallCtx(const Context *ctx) {
    bg_ctx c;
    c.now_ns = ctx->current_ns;
    c.igate = ctx->current_igate;
    c.device = -1;
    c.wid = (uint32_t)ctx->wid;
    return c;
  }

  // ProcessBatch on the GPU, synchronously
  void Forward(Context *ctx, bess::PacketBatch *batch) {
    const int n = batch->cnt();
    uint8_t *heads[bess::PacketBatch::kMaxBurst] = {};
    uint16_t og[bess::PacketBatch::kMaxBurst];
    for (int i = 0; i < n; i++) heads[i] = batch->pkts()[i]->head_data<uint8_t *>();
    const bg_ctx c = CallCtx(ctx);
    if (bg_module_process(m_, &c, heads, (size_t)n, og) < 0) {
      for (int i = 0; i < n; i++) DropPacket(ctx, batch->pkts()[i]);
      return;
    }
    Emit(ctx, batch, og);
  }

  // a gate per packet: BG_GATE_NONE leaves the packet alone (the module did
  // not emit it), BG_DROP_GATE drops it, any other gate goes to EmitPacket
  void Emit(Context *ctx, bess::PacketBatch *batch, const uint16_t *og) {
    for (int i = 0; i < batch->cnt(); i++) {
      bess::Packet *pkt = batch->pkts()[i];
      if (og[i] == BG_GATE_NONE) continue;
      if (og[i] >= BG_MAX_GATES)
        DropPacket(ctx, pkt);
      else
        EmitPacket(ctx, pkt, og[i]);
    }
  }

  std::string Desc() const {
    char b[256] = "";
    if (m_) bg_module_desc(m_, b, sizeof(b));
    return b;
  }

  bg_module *m_ = nullptr;
};

#endif  // BESS_MODULES_GPU_MODULE_H_
