// module.cc -- module registry, command responses and the bg_module_* C ABI
// (include/bessgpu.h), i.e. what core/module.cc + core/bessctl.cc's
// CreateModule / ModuleCommand do for a module, minus gRPC.
#include "module.h"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <mutex>

#include "../../include/bessgpu.h"
#include "../csrc/bg_internal.h"

CommandResponse CommandSuccess() { return CommandResponse(); }

CommandResponse CommandSuccess(const bess::pb::Message &m) {
  CommandResponse r;
  r.set_data(m.SerializeAsString());
  return r;
}

CommandResponse CommandFailure(int code, const char *fmt, ...) {
  CommandResponse r;
  std::string msg;
  if (fmt) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    msg = buf;
  }
  r.set_error(code, msg);
  return r;
}

namespace {
std::map<std::string, ModuleBuilder> &builders() {
  static std::map<std::string, ModuleBuilder> m;
  return m;
}
}  // namespace

bool ModuleBuilder::RegisterModuleClass(const std::string &class_name,
                                        const std::string &name_template,
                                        const std::string &help, Factory f) {
  ModuleBuilder b;
  b.name_template_ = name_template;
  b.help_ = help;
  b.factory_ = std::move(f);
  // first registration of a class name wins (core/module.cc:46-57)
  return builders().emplace(class_name, std::move(b)).second;
}

const ModuleBuilder *ModuleBuilder::Find(const std::string &class_name) {
  auto it = builders().find(class_name);
  return it == builders().end() ? nullptr : &it->second;
}

std::vector<std::string> ModuleBuilder::Classes() {
  std::vector<std::string> v;
  for (auto &kv : builders()) v.push_back(kv.first);
  return v;
}

using bg::fail;

static int respond(const CommandResponse &r) {
  if (r.code() != 0) return fail(r.code(), "%s", r.errmsg().c_str());
  bg::g_err.clear();
  return 0;
}

extern "C" {

int bg_module_create(const char *mclass, const void *arg, size_t arg_len,
                     bg_module **out) {
  const ModuleBuilder *b = ModuleBuilder::Find(mclass ? mclass : "");
  if (!b) return fail(ENOENT, "No module class '%s' found", mclass ? mclass : "");
  std::unique_ptr<Module> m;
  CommandResponse r = b->Create(arg, arg_len, &m);
  if (r.code() != 0) return respond(r);
  bg_module *h = new bg_module();
  h->m = std::move(m);
  h->mclass = mclass;
  *out = h;
  return 0;
}

void bg_module_destroy(bg_module *m) { delete m; }

// ModuleBuilder::RunCommand (core/module.cc:92-116)
int bg_module_command(bg_module *h, const char *cmd, const void *arg,
                      size_t arg_len, void *out, size_t *out_len) {
  std::lock_guard<std::mutex> lk(h->mu);
  const std::string user_cmd = cmd ? cmd : "";
  for (const Command &c : h->m->cmds()) {
    if (c.cmd != user_cmd) continue;
    CommandResponse r = c.func(h->m.get(), arg, arg_len);
    if (r.code() != 0) return respond(r);
    const std::string &d = r.data();
    if (out_len) {
      size_t cap = *out_len;
      *out_len = d.size();
      if (out && cap >= d.size()) memcpy(out, d.data(), d.size());
      else if (d.size() > cap)
        return fail(ENOBUFS, "response needs %zu bytes", d.size());
    }
    bg::g_err.clear();
    return 0;
  }
  return fail(ENOTSUP, "'%s' does not support command '%s'", h->mclass.c_str(),
              user_cmd.c_str());
}

int bg_module_process(bg_module *h, uint8_t *const *heads, size_t cnt,
                      uint16_t *ogates) {
  std::lock_guard<std::mutex> lk(h->mu);
  for (size_t i = 0; i < cnt; i++) ogates[i] = BG_GATE_NONE;
  std::vector<bess::Packet> pkts(cnt);
  std::vector<bess::Packet *> ptrs(cnt);
  for (size_t i = 0; i < cnt; i++) {
    pkts[i] = bess::Packet(heads[i], 2048, (uint32_t)i);  // SNBUF_DATA span
    ptrs[i] = &pkts[i];
  }
  Context ctx;
  ctx.ogates = ogates;
  bg::g_err.clear();
  int r = h->m->ProcessPackets(&ctx, ptrs.data(), cnt);
  return r;
}

int bg_module_process_device(bg_module *h, void *d_frames, size_t stride,
                             size_t n, uint16_t *d_ogates, bg_stream_t stream) {
  return h->m->ProcessDevice(d_frames, stride, n, d_ogates, stream);
}

int bg_module_set_device(bg_module *h, int device) {
  h->m->set_device(device);
  return 0;
}

int bg_module_set_igate(bg_module *h, uint16_t igate) {
  h->m->set_igate(igate);
  return 0;
}

int bg_module_bind_meta(bg_module *h, int meta_off, const char *const *names,
                        const int32_t *offsets, int n) {
  if (n < 0 || (n > 0 && (!names || !offsets))) return fail(EINVAL, "bad arguments");
  std::vector<std::string> nm;
  std::vector<int32_t> off;
  for (int i = 0; i < n; i++) {
    nm.emplace_back(names[i] ? names[i] : "");
    off.push_back(offsets[i]);
  }
  std::lock_guard<std::mutex> lk(h->mu);
  bg::g_err.clear();
  int r = h->m->BindMeta(meta_off, nm, off);
  if (r == -ENOTSUP && bg::g_err.empty())
    return fail(ENOTSUP, "'%s' has no metadata fields on its datapath",
                h->mclass.c_str());
  return r;
}

int bg_module_desc(const bg_module *h, char *buf, size_t len) {
  std::string d = h->m->GetDesc();
  if (buf && len) {
    snprintf(buf, len, "%s", d.c_str());
  }
  return (int)d.size();
}

}  // extern "C"
