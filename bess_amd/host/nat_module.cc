// nat_module.cc -- NAT (core/modules/nat.{h,cc}): dynamic address/port
// translation with its ProcessBatch on the GPU (bg_dnat_*, bg_dnat.hip).
// Same class name, commands table, Init argument, error codes and
// messages; two input gates (each call's input gate, bg_ctx::igate, picks
// the direction) and the call's ctx->current_ns (bg_ctx::now_ns) as the
// mapping clock.
#include <errno.h>
#include <stdio.h>
#include <time.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "module.h"

using bess::pb::EmptyArg;
using bess::pb::NATArg;

namespace {

bool ParseIpv4(const std::string &str, uint32_t *addr) {  // core/utils/ip.cc:40-51
  unsigned a, b, c, d;
  if (sscanf(str.c_str(), "%u.%u.%u.%u", &a, &b, &c, &d) != 4 || a >= 256 ||
      b >= 256 || c >= 256 || d >= 256)
    return false;
  *addr = (a << 24) | (b << 16) | (c << 8) | d;
  return true;
}

std::string ToIpv4(uint32_t a) {  // ip.cc:53-61
  char buf[20];
  snprintf(buf, sizeof(buf), "%u.%u.%u.%u", a >> 24, (a >> 16) & 255,
           (a >> 8) & 255, a & 255);
  return buf;
}

}  // namespace

class NAT final : public Module {
 public:
  static const gate_idx_t kNumIGates = 2;
  static const gate_idx_t kNumOGates = 2;
  static const Commands kCmds;

  ~NAT() override { bg_dnat_destroy(h_); }

  const Commands &cmds() const override { return kCmds; }

  // nat.cc:65-113: bg_dnat_create checks the ranges and addresses with the
  // reference's messages; kept here for GetInitialArg: the addresses sorted
  // (nat.cc:110), the port lists in argument order, as the reference does
  CommandResponse Init(const NATArg &arg) {
    std::vector<std::string> addrs;
    std::vector<const char *> ap;
    std::vector<int32_t> nr;
    std::vector<int64_t> b, e;
    std::vector<uint8_t> su;
    for (const auto &x : arg.ext_addrs()) {
      addrs.push_back(x.ext_addr());
      nr.push_back(x.port_ranges().size());
      for (const auto &r : x.port_ranges()) {
        b.push_back(r.begin());
        e.push_back(r.end());
        su.push_back(r.suspended() ? 1 : 0);
      }
    }
    for (auto &s : addrs) ap.push_back(s.c_str());
    int rc = bg_dnat_create(ap.data(), (int)ap.size(), nr.data(), b.data(), e.data(),
                            su.data(), (uint64_t)time(nullptr), &h_);
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    size_t k = 0;
    for (size_t i = 0; i < addrs.size(); i++) {
      uint32_t a = 0;
      ParseIpv4(addrs[i], &a);
      ext_addrs_.push_back(a);
      std::vector<Range> pl;
      if (nr[i] == 0) pl.push_back({0, 65535, false});
      for (int32_t j = 0; j < nr[i]; j++, k++)
        pl.push_back({(uint16_t)b[k], (uint16_t)e[k], su[k] != 0});
      ranges_.push_back(pl);
    }
    std::sort(ext_addrs_.begin(), ext_addrs_.end());
    return CommandSuccess();
  }

  // nat.cc:115-128
  CommandResponse GetInitialArg(const EmptyArg &) {
    NATArg resp;
    for (size_t i = 0; i < ext_addrs_.size(); i++) {
      auto *ext = resp.add_ext_addrs();
      ext->set_ext_addr(ToIpv4(ext_addrs_[i]));
      for (const auto &r : ranges_[i]) {
        auto *pr = ext->add_port_ranges();
        pr->set_begin(r.begin);
        pr->set_end(r.end);
        pr->set_suspended(r.suspended);
      }
    }
    return CommandSuccess(resp);
  }
  CommandResponse GetRuntimeConfig(const EmptyArg &) { return CommandSuccess(); }
  CommandResponse SetRuntimeConfig(const EmptyArg &) { return CommandSuccess(); }

  // nat.cc:377-380
  std::string GetDesc() const override {
    char b[64];
    snprintf(b, sizeof(b), "%zu entries", bg_dnat_count(h_));
    return b;
  }

  // DoProcessBatch<dir> (nat.cc:321-363). The mapping table is the
  // module's state: batches go through it one at a time.
  int ProcessDevice(const bg_ctx &c, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    std::lock_guard<std::mutex> g(mu_);
    return bg_dnat_process(h_, d_frames, stride, n, c.igate ? 1 : 0, c.now_ns,
                           d_ogates, stream);
  }
  unsigned CtxUse() const override { return kCtxIgate | kCtxNow; }

  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    *lo = 0;
    *hi = 128;  // Ethernet + IPv4 (any IHL) + the L4 ports and checksum
    *writeback = true;
  }

 private:
  struct Range {
    uint16_t begin, end;
    bool suspended;
  };
  std::vector<uint32_t> ext_addrs_;
  std::vector<std::vector<Range>> ranges_;
  bg_dnat *h_ = nullptr;
  std::mutex mu_;
};

const Commands NAT::kCmds = {
    {"get_initial_arg", "EmptyArg", MODULE_CMD_FUNC(&NAT::GetInitialArg),
     Command::THREAD_SAFE},
    {"get_runtime_config", "EmptyArg", MODULE_CMD_FUNC(&NAT::GetRuntimeConfig),
     Command::THREAD_SAFE},
    {"set_runtime_config", "EmptyArg", MODULE_CMD_FUNC(&NAT::SetRuntimeConfig),
     Command::THREAD_SAFE}};

ADD_MODULE_ARG(NAT, bess::pb::NATArg, "nat", "Dynamic Network address/port translator")
