// acl_module.cc -- ACL (core/modules/acl.{h,cc}) with its ProcessBatch on
// the GPU (bg_acl_*, bg_acl.hip). Same class name, commands table, Init
// argument and rule semantics (Ipv4Prefix parsing, port 0 = wildcard,
// first match decides, "established" ignored). One deliberate difference:
// a prefix length that std::stoi cannot parse throws in the reference
// (ip.cc:77, never caught); here the command fails with EINVAL.
#include <errno.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "module.h"

using bess::pb::ACLArg;
using bess::pb::ACLArg_Rule;
using bess::pb::EmptyArg;

namespace {

// Ipv4Prefix::Ipv4Prefix (core/utils/ip.cc:63-79) with ParseIpv4Address
// (40-51); false where std::stoi would throw.
bool ParseIpv4Prefix(const std::string &prefix, uint32_t *addr, uint32_t *mask) {
  *addr = 0;
  *mask = 0;
  const size_t delim = prefix.find('/');
  if (prefix.empty() || delim == std::string::npos || delim >= prefix.size())
    return true;
  unsigned a, b, c, d;
  const std::string ip = prefix.substr(0, delim);
  if (sscanf(ip.c_str(), "%u.%u.%u.%u", &a, &b, &c, &d) == 4 && a < 256 &&
      b < 256 && c < 256 && d < 256)
    *addr = (a << 24) | (b << 16) | (c << 8) | d;
  const std::string ls = prefix.substr(delim + 1);
  const char *s = ls.c_str();
  char *end = nullptr;
  errno = 0;
  const long v = strtol(s, &end, 10);
  if (end == s || errno == ERANGE || v > INT_MAX || v < INT_MIN) return false;
  const size_t n = (size_t)(long)(int)v;  // SetBitsLow<uint32_t>(size_t(len))
  *mask = n == 0 ? 0u : n >= 32 ? 0xFFFFFFFFu : ~((1u << (32 - n)) - 1u);
  return true;
}

}  // namespace

class ACL final : public Module {
 public:
  static const Commands kCmds;

  ~ACL() override { bg_acl_destroy(h_); }

  const Commands &cmds() const override { return kCmds; }

  // acl.cc:42-53
  CommandResponse Init(const ACLArg &arg) {
    if (!h_) {
      int rc = bg_acl_create(&h_);
      if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    }
    std::vector<bg_acl_rule> add;
    for (const ACLArg_Rule &r : arg.rules()) {
      bg_acl_rule x;
      memset(&x, 0, sizeof(x));
      if (!ParseIpv4Prefix(r.src_ip(), &x.src_addr, &x.src_mask) ||
          !ParseIpv4Prefix(r.dst_ip(), &x.dst_addr, &x.dst_mask))
        return CommandFailure(EINVAL, "invalid prefix length");
      x.src_port = (uint16_t)r.src_port();
      x.dst_port = (uint16_t)r.dst_port();
      x.drop = r.drop() ? 1 : 0;
      add.push_back(x);
    }
    int rc = bg_acl_add(h_, add.data(), add.size());
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    return CommandSuccess();
  }

  // acl.cc:55-58
  CommandResponse CommandAdd(const ACLArg &arg) {
    Init(arg);
    return CommandSuccess();
  }

  // acl.cc:60-63
  CommandResponse CommandClear(const EmptyArg &) {
    bg_acl_clear(h_);
    return CommandSuccess();
  }

  // acl.cc:70: a packet the first matching rule forwards leaves on the
  // input gate it came in on -- the call's, ctx->current_igate
  int ProcessDevice(const bg_ctx &c, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    return bg_acl_classify(h_, d_frames, stride, n, c.igate, d_ogates, stream);
  }
  unsigned CtxUse() const override { return kCtxIgate; }

  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    *lo = 0;
    *hi = 80;
    *writeback = false;
  }

 private:
  bg_acl *h_ = nullptr;
};

const Commands ACL::kCmds = {
    {"add", "ACLArg", MODULE_CMD_FUNC(&ACL::CommandAdd), Command::THREAD_UNSAFE},
    {"clear", "EmptyArg", MODULE_CMD_FUNC(&ACL::CommandClear),
     Command::THREAD_UNSAFE}};

ADD_MODULE_ARG(ACL, bess::pb::ACLArg, "acl", "ACL module from NetBricks")
