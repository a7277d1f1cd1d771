// static_nat_module.cc -- StaticNAT (core/modules/static_nat.{h,cc}) with
// its ProcessBatch on the GPU (bg_snat_*, bg_nat.hip). Same class name,
// commands table, Init argument, error codes and messages; two input gates
// (the input gate of each call, bg_ctx::igate, picks the direction).
#include <errno.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "module.h"

using bess::pb::EmptyArg;
using bess::pb::StaticNATArg;

namespace {

// ParseIpv4Address (core/utils/ip.cc:40-51)
bool ParseIpv4Address(const std::string &str, uint32_t *addr) {
  unsigned a, b, c, d;
  if (sscanf(str.c_str(), "%u.%u.%u.%u", &a, &b, &c, &d) != 4 || a >= 256 ||
      b >= 256 || c >= 256 || d >= 256)
    return false;
  *addr = (a << 24) | (b << 16) | (c << 8) | d;
  return true;
}

// ToIpv4Address (ip.cc:53-61)
std::string ToIpv4Address(uint32_t a) {
  char buf[20];
  snprintf(buf, sizeof(buf), "%u.%u.%u.%u", a >> 24, (a >> 16) & 255,
           (a >> 8) & 255, a & 255);
  return buf;
}

}  // namespace

class StaticNAT final : public Module {
 public:
  static const gate_idx_t kNumIGates = 2;
  static const gate_idx_t kNumOGates = 2;
  static const Commands kCmds;

  ~StaticNAT() override { bg_snat_destroy(h_); }

  const Commands &cmds() const override { return kCmds; }

  // static_nat.cc:44-91
  CommandResponse Init(const StaticNATArg &arg) {
    int rc = bg_snat_create(&h_);
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    for (const auto &p : arg.pairs()) {
      uint32_t is, ie, es, ee;
      if (!ParseIpv4Address(p.int_range().start(), &is))
        return CommandFailure(EINVAL, "invalid IP address %s",
                              p.int_range().start().c_str());
      if (!ParseIpv4Address(p.int_range().end(), &ie))
        return CommandFailure(EINVAL, "invalid IP address %s",
                              p.int_range().end().c_str());
      if (is > ie) return CommandFailure(EINVAL, "invalid internal IP address range");
      if (!ParseIpv4Address(p.ext_range().start(), &es))
        return CommandFailure(EINVAL, "invalid IP address %s",
                              p.ext_range().start().c_str());
      if (!ParseIpv4Address(p.ext_range().end(), &ee))
        return CommandFailure(EINVAL, "invalid IP address %s",
                              p.ext_range().end().c_str());
      if (es > ee) return CommandFailure(EINVAL, "invalid external IP address range");
      if (ie == 0xffffffffu || ee == 0xffffffffu)
        return CommandFailure(EINVAL, "cannot map broadcast address");
      if (ie - is != ee - es)
        return CommandFailure(EINVAL, "internal/external address ranges differ");
      pairs_.push_back({is, es, ie - is + 1});
      bg_snat_add(h_, is, es, ie - is + 1);
    }
    return CommandSuccess();
  }

  // static_nat.cc:93-111 (the end it reports is start + size)
  CommandResponse GetInitialArg(const EmptyArg &) {
    StaticNATArg resp;
    for (const auto &p : pairs_) {
      auto *pb = resp.add_pairs();
      pb->mutable_int_range()->set_start(ToIpv4Address(p.int_addr));
      pb->mutable_int_range()->set_end(ToIpv4Address(p.int_addr + p.size));
      pb->mutable_ext_range()->set_start(ToIpv4Address(p.ext_addr));
      pb->mutable_ext_range()->set_end(ToIpv4Address(p.ext_addr + p.size));
    }
    return CommandSuccess(resp);
  }
  CommandResponse GetRuntimeConfig(const EmptyArg &) { return CommandSuccess(); }
  CommandResponse SetRuntimeConfig(const EmptyArg &) { return CommandSuccess(); }

  // static_nat.cc:146-181: input gate 0 translates the source, 1 the
  // destination -- the call's gate, ctx->current_igate
  int ProcessDevice(const bg_ctx &c, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    return bg_snat_classify(h_, d_frames, stride, n, c.igate ? 1 : 0, d_ogates,
                            stream);
  }
  unsigned CtxUse() const override { return kCtxIgate; }

  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    *lo = 0;
    *hi = 128;  // the L4 checksum of any IHL lies below byte 128
    *writeback = true;
  }

 private:
  struct NatPair {
    uint32_t int_addr, ext_addr, size;
  };
  std::vector<NatPair> pairs_;
  bg_snat *h_ = nullptr;
};

const Commands StaticNAT::kCmds = {
    {"get_initial_arg", "EmptyArg", MODULE_CMD_FUNC(&StaticNAT::GetInitialArg),
     Command::THREAD_SAFE},
    {"get_runtime_config", "EmptyArg",
     MODULE_CMD_FUNC(&StaticNAT::GetRuntimeConfig), Command::THREAD_SAFE},
    {"set_runtime_config", "EmptyArg",
     MODULE_CMD_FUNC(&StaticNAT::SetRuntimeConfig), Command::THREAD_SAFE}};

ADD_MODULE_ARG(StaticNAT, bess::pb::StaticNATArg, "static_nat",
               "Static network address translator")
