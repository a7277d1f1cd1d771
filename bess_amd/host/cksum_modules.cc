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

  // the whole frame goes to the device; the recomputed checksum words come
  // back (bg_pipe writes the header line back into the packet buffer)
  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    *lo = 0;
    *hi = 2048;
    *writeback = true;
  }

  int ProcessDevice(const bg_ctx &c, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    return bg_cksum(c.device, d_frames, stride, n, kMode, verify_ ? 1 : 0,
                    kMode == BG_CK_IP ? d_ogates : nullptr,
                    kMode == BG_CK_L4 ? d_ogates : nullptr, stream);
  }

 private:
  bool verify_ = false;
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
