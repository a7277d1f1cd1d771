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

  // The bytes the reference reads past data_len (P11): L4Checksum sums
  // udp.length bytes from the UDP header (checksum.h:398-407) or ip.length
  // minus the IP header from the TCP header (checksum.h:492-504) of an
  // untagged IPv4 frame (l4_checksum.cc:53-82), without checking data_len.
  // IPChecksum reads at most 22 + 60 bytes, inside the header line the pipe
  // always stages.
  size_t StageReach(const uint8_t *f, size_t len) const override {
    if (kMode != BG_CK_L4 || f[12] != 0x08 || f[13] != 0x00) return len;
    const size_t l4 = 14 + (size_t)(f[14] & 15) * 4;
    size_t end = 0;
    if (f[23] == 17) {  // UDP: length at l4 + 4 (l4 + 6 <= 80, in the line)
      const size_t ulen = (size_t)f[l4 + 4] << 8 | f[l4 + 5];
      if (ulen >= 8) end = l4 + ulen;
    } else if (f[23] == 6) {  // TCP: ip.length - IHL*4 bytes from l4
      const size_t ip_len = (size_t)f[16] << 8 | f[17];
      if (ip_len >= l4 - 14 + 20) end = 14 + ip_len;
    }
    return std::max(len, end);
  }

  int ProcessDevice(const bg_ctx &c, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    return bg_cksum(c.device, d_frames, stride, n, kMode, verify_ ? 1 : 0,
                    kMode == BG_CK_IP ? d_ogates : nullptr,
                    kMode == BG_CK_L4 ? d_ogates : nullptr, stream);
  }

  // the frames in place (host-registered packet buffers): no staging copy
  int ProcessDevicePtrs(const bg_ctx &c, const uint64_t *d_ptrs, size_t span, size_t n,
                        uint16_t *d_ogates, void *stream) override {
    if (n == 0) return 0;
    return bg_cksum_ptrs(c.device, d_ptrs, span, n, kMode, verify_ ? 1 : 0,
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
