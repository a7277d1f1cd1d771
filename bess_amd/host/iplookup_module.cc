// iplookup_module.cc -- IPLookup (core/modules/ip_lookup.{h,cc}) with its
// ProcessBatch on the GPU (bg_lpm_*, bg_lpm.hip). Same class name, commands
// table, Init argument, error codes and messages; prefix_len 0 sets /
// resets the default gate as in the reference.
#include <errno.h>
#include <inttypes.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "module.h"

using bess::pb::EmptyArg;
using bess::pb::IPLookupArg;
using bess::pb::IPLookupCommandAddArg;
using bess::pb::IPLookupCommandDeleteArg;

class IPLookup final : public Module {
 public:
  static const gate_idx_t kNumOGates = MAX_GATES;
  static const Commands kCmds;

  ~IPLookup() override { bg_lpm_destroy(lpm_); }

  const Commands &cmds() const override { return kCmds; }

  // ip_lookup.cc:54-69
  CommandResponse Init(const IPLookupArg &arg) {
    default_gate_ = DROP_GATE;
    int rc = bg_lpm_create(arg.max_rules() ? arg.max_rules() : 1024,
                           arg.max_tbl8s() ? arg.max_tbl8s() : 128, &lpm_);
    if (rc < 0) return CommandFailure(-rc, "DPDK error: %s", bg_last_error());
    return CommandSuccess();
  }

  // ip_lookup.cc:153-184 ParseIpv4Prefix
  static int ParseIpv4Prefix(const std::string &prefix, uint64_t prefix_len,
                             std::string *err, uint32_t *net_addr) {
    char buf[160];
    if (!prefix.length()) {
      *err = "prefix' is missing";
      return EINVAL;
    }
    unsigned a, b, c, d;
    // ParseIpv4Address (core/utils/ip.cc:40-51)
    if (sscanf(prefix.c_str(), "%u.%u.%u.%u", &a, &b, &c, &d) != 4 || a >= 256 ||
        b >= 256 || c >= 256 || d >= 256) {
      snprintf(buf, sizeof(buf), "Invalid IP prefix: %s", prefix.c_str());
      *err = buf;
      return EINVAL;
    }
    const uint32_t addr = (a << 24) | (b << 16) | (c << 8) | d;
    if (prefix_len > 32) {
      snprintf(buf, sizeof(buf), "Invalid prefix length: %" PRIu64, prefix_len);
      *err = buf;
      return EINVAL;
    }
    const uint32_t mask = prefix_len == 0 ? 0u
                          : prefix_len >= 32 ? 0xFFFFFFFFu
                                             : ~((1u << (32 - prefix_len)) - 1u);
    if (addr & ~mask) {
      snprintf(buf, sizeof(buf), "Invalid IP prefix %s/%" PRIu64 " %x %x",
               prefix.c_str(), prefix_len, addr, mask);
      *err = buf;
      return EINVAL;
    }
    *net_addr = addr;
    return 0;
  }

  // ip_lookup.cc:186-211
  CommandResponse CommandAdd(const IPLookupCommandAddArg &arg) {
    const gate_idx_t gate = (gate_idx_t)arg.gate();
    const uint64_t prefix_len = arg.prefix_len();
    std::string err;
    uint32_t net_addr = 0;
    int e = ParseIpv4Prefix(arg.prefix(), prefix_len, &err, &net_addr);
    if (e) return CommandFailure(e, "%s", err.c_str());
    if (!(gate < MAX_GATES || gate == DROP_GATE))
      return CommandFailure(EINVAL, "Invalid gate: %hu", gate);
    if (prefix_len == 0) {
      default_gate_ = gate;
    } else {
      int ret = bg_lpm_add(lpm_, net_addr, (int)prefix_len, gate);
      if (ret) return CommandFailure(-ret, "rpm_lpm_add() failed");
    }
    return CommandSuccess();
  }

  // ip_lookup.cc:213-233
  CommandResponse CommandDelete(const IPLookupCommandDeleteArg &arg) {
    const uint64_t prefix_len = arg.prefix_len();
    std::string err;
    uint32_t net_addr = 0;
    int e = ParseIpv4Prefix(arg.prefix(), prefix_len, &err, &net_addr);
    if (e) return CommandFailure(e, "%s", err.c_str());
    if (prefix_len == 0) {
      default_gate_ = DROP_GATE;
    } else {
      int ret = bg_lpm_delete(lpm_, net_addr, (int)prefix_len);
      if (ret) return CommandFailure(-ret, "rpm_lpm_delete() failed");
    }
    return CommandSuccess();
  }

  // ip_lookup.cc:235-238
  CommandResponse CommandClear(const EmptyArg &) {
    bg_lpm_clear(lpm_);
    return CommandSuccess();
  }

  int ProcessDevice(const bg_ctx &, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    return bg_lpm_classify(lpm_, d_frames, stride, n, default_gate_, d_ogates,
                           stream);
  }

  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    *lo = 0;
    *hi = 64;
    *writeback = false;
  }

 private:
  bg_lpm *lpm_ = nullptr;
  gate_idx_t default_gate_ = DROP_GATE;
};

const Commands IPLookup::kCmds = {
    {"add", "IPLookupCommandAddArg", MODULE_CMD_FUNC(&IPLookup::CommandAdd),
     Command::THREAD_UNSAFE},
    {"delete", "IPLookupCommandDeleteArg",
     MODULE_CMD_FUNC(&IPLookup::CommandDelete), Command::THREAD_UNSAFE},
    {"clear", "EmptyArg", MODULE_CMD_FUNC(&IPLookup::CommandClear),
     Command::THREAD_UNSAFE}};

ADD_MODULE_ARG(IPLookup, bess::pb::IPLookupArg, "ip_lookup",
               "performs Longest Prefix Match on IPv4 packets")
