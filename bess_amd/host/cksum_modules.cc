// cksum_modules.cc -- IPChecksum and L4Checksum (core/modules/ip_checksum.cc,
// l4_checksum.cc) with their ProcessBatch on the GPU (bg_cksum*,
// bg_kernels.hip cksum_kernel). Output gates: 0 forward, 1 fail; packets the
// reference never emits (L4Checksum: TCP in recompute mode, IPv4 that is
// neither UDP nor TCP) get no gate.
#include <algorithm>
#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "module.h"

namespace {

template <int kMode>
class ChecksumModule : public Module {
 public:
  static const gate_idx_t kNumOGates = 2;  // (0) forward, (1) fail
  static const Commands kCmds;

  const Commands &cmds() const override { return kCmds; }

  // ip_checksum.cc:86-89 / l4_checksum.cc:85-88
  CommandResponse Init(const bess::pb::VerifyArg &arg) {
    verify_ = arg.verify();
    return CommandSuccess();
  }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override {
    ProcessPackets(ctx, batch->pkts(), (size_t)batch->cnt());
  }

  int ProcessPackets(Context *ctx, bess::Packet *const *pkts,
                     size_t cnt) override {
    if (cnt == 0) return 0;
    heads_.resize(cnt);
    gates_.resize(cnt);
    uint32_t span = 0xFFFFFFFFu;
    for (size_t i = 0; i < cnt; i++) {
      heads_[i] = pkts[i]->head_data<uint8_t *>();
      span = std::min(span, pkts[i]->span());
    }
    uint16_t *ipg = kMode == BG_CK_IP ? gates_.data() : nullptr;
    uint16_t *l4g = kMode == BG_CK_L4 ? gates_.data() : nullptr;
    int rc = bg_cksum_process_host(device_, heads_.data(), cnt, span, kMode,
                                   verify_ ? 1 : 0, ipg, l4g, nullptr);
    if (rc < 0) {
      for (size_t i = 0; i < cnt; i++) DropPacket(ctx, pkts[i]);
      return rc;
    }
    for (size_t i = 0; i < cnt; i++)
      if (gates_[i] != BG_GATE_NONE) EmitPacket(ctx, pkts[i], gates_[i]);
    return 0;
  }

  // the whole frame goes to the device; the recomputed checksum words come
  // back (bg_pipe writes the header line back into the packet buffer)
  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    *lo = 0;
    *hi = 2048;
    *writeback = true;
  }

  int ProcessDevice(void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    return bg_cksum(device_, d_frames, stride, n, kMode, verify_ ? 1 : 0,
                    kMode == BG_CK_IP ? d_ogates : nullptr,
                    kMode == BG_CK_L4 ? d_ogates : nullptr, stream);
  }

 private:
  bool verify_ = false;
  std::vector<uint8_t *> heads_;
  std::vector<uint16_t> gates_;
};

template <int kMode>
const Commands ChecksumModule<kMode>::kCmds = {};

}  // namespace

class IPChecksum final : public ChecksumModule<BG_CK_IP> {};
class L4Checksum final : public ChecksumModule<BG_CK_L4> {};

ADD_MODULE_ARG(IPChecksum, bess::pb::IPChecksumArg, "ip_checksum",
               "recomputes the IPv4 checksum")
ADD_MODULE_ARG(L4Checksum, bess::pb::L4ChecksumArg, "l4_checksum",
               "recomputes the TCP/Ipv4 and UDP/IPv4 checksum")
