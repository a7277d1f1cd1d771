// module.cc -- module registry, command responses and the bg_module_* C ABI
// (include/bessgpu.h), i.e. what core/module.cc + core/bessctl.cc's
// CreateModule / ModuleCommand do for a module, minus gRPC.
#include "module.h"

#include <stdio.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <shared_mutex>

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

// A call's context with its defaults filled in (bg_ctx, include/bessgpu.h):
// no ctx = input gate 0 and the monotonic clock now; device -1 = the
// module's.
bg_ctx ResolveCtx(const bg_ctx *c, int module_device) {
  bg_ctx r{};
  if (c) {
    r = *c;
  } else {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    r.now_ns = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
  }
  if (r.device < 0) r.device = (int16_t)module_device;
  return r;
}

// The synchronous host datapath shared by every module (see module.h).
int Module::ProcessPackets(Context *ctx, bess::Packet *const *pkts, size_t cnt) {
  if (cnt == 0) return 0;
  int lo, hi, mlo, mhi;
  bool wb;
  DeviceWindow(&lo, &hi, &wb);
  auto drop_all = [&](int rc) {
    for (size_t i = 0; i < cnt; i++) DropPacket(ctx, pkts[i]);
    return rc;
  };
  int r = MetaWindow(&mlo, &mhi);
  if (r) return drop_all(r);
  const bool meta = mhi > mlo;  // attr fields: the row carries metadata too
  if (meta)
    for (size_t i = 0; i < cnt; i++)
      if (!pkts[i]->metadata<uint8_t *>())
        return drop_all(fail(EINVAL, "the module reads metadata attributes: "
                             "pass each packet's metadata area"));
  uint32_t span = 0xFFFFFFFFu;
  for (size_t i = 0; i < cnt; i++) span = std::min(span, pkts[i]->span());
  if (!meta && hi > (int)span) hi = (int)span;
  if (hi <= lo) hi = lo + 1;
  const size_t len = (size_t)(hi - lo);
  const size_t w = meta ? StagedStride(lo, hi, mlo, mhi) : (len + 15) / 16 * 16;
  const size_t mat = (size_t)StagedMetaAt(lo, hi), mlen = (size_t)(mhi - mlo);
  const size_t line = std::min<size_t>(w, 128);  // header line written back
  const bg_ctx &c = ctx->call;
  r = bg::set_device(c.device);
  if (r) return drop_all(r);
  bg::Staging &st = bg::thread_staging();
  // +64 B: the last window's 16-byte loads may run past its slot
  r = st.ensure(c.device, cnt * w + 64, cnt * 2);
  if (r) return drop_all(r);
  hipStream_t s = bg::thread_stream(c.device, nullptr);
  for (size_t i = 0; i < cnt; i++) {
    uint8_t *dst = st.h_in + i * w;
    memcpy(dst, pkts[i]->head_data<uint8_t *>() + lo, len);
    if (w > len) memset(dst + len, 0, w - len);
    if (meta) memcpy(dst + mat, pkts[i]->metadata<uint8_t *>() + mlo, mlen);
  }
  uint16_t *d_g = reinterpret_cast<uint16_t *>(st.d_out);
  hipError_t e = hipMemcpyAsync(st.d_in, st.h_in, cnt * w, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return drop_all(fail(EIO, "H2D: %s", hipGetErrorString(e)));
  r = ProcessDeviceWindow(c, st.d_in, w, cnt, lo, d_g, s);
  if (r < 0) {
    (void)hipStreamSynchronize(s);
    return drop_all(r);
  }
  e = hipMemcpyAsync(st.h_out, d_g, cnt * 2, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && wb)
    e = hipMemcpy2DAsync(st.h_in, line, st.d_in, w, line, cnt,
                         hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return drop_all(fail(EIO, "D2H: %s", hipGetErrorString(e)));
  const uint16_t *g = reinterpret_cast<const uint16_t *>(st.h_out);
  for (size_t i = 0; i < cnt; i++) {
    if (wb && lo == 0)
      memcpy(pkts[i]->head_data<uint8_t *>(), st.h_in + i * line,
             std::min(line, len));
    if (g[i] != BG_GATE_NONE) EmitPacket(ctx, pkts[i], g[i]);
  }
  return 0;
}

void ModuleUnref(bg_module *m) {
  if (m->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete m;
}

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

void bg_module_destroy(bg_module *m) {
  if (m) ModuleUnref(m);
}

// ModuleBuilder::RunCommand (core/module.cc:92-116)
int bg_module_command(bg_module *h, const char *cmd, const void *arg,
                      size_t arg_len, void *out, size_t *out_len) {
  const std::string user_cmd = cmd ? cmd : "";
  for (const Command &c : h->m->cmds()) {
    if (c.cmd != user_cmd) continue;
    std::shared_lock<std::shared_mutex> shared(h->mu, std::defer_lock);
    std::unique_lock<std::shared_mutex> excl(h->mu, std::defer_lock);
    if (c.mt_safe == Command::THREAD_SAFE) {
      shared.lock();
    } else {
      excl.lock();
      // batches submitted before a rule change keep the rules they were
      // submitted under: their partly filled pipe slots launch now, and the
      // device images they read are retired behind fences (bg_image.h)
      std::lock_guard<std::mutex> pl(h->pipes_mu);
      for (bg_pipe *p : h->pipes)
        if (int r = PipeFlushLocked(p)) return r;
    }
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

static int process(bg_module *h, const bg_ctx *call, uint8_t *const *heads,
                   uint8_t *const *metas, size_t cnt, uint16_t *ogates, EmitLog *log) {
  std::shared_lock<std::shared_mutex> lk(h->mu);  // many workers at once
  for (size_t i = 0; i < cnt; i++) ogates[i] = BG_GATE_NONE;
  std::vector<bess::Packet> pkts(cnt);
  std::vector<bess::Packet *> ptrs(cnt);
  for (size_t i = 0; i < cnt; i++) {
    pkts[i] = bess::Packet(heads[i], 2048, (uint32_t)i,  // SNBUF_DATA span
                           metas ? metas[i] : nullptr);
    ptrs[i] = &pkts[i];
  }
  Context ctx;
  ctx.call = ResolveCtx(call, h->m->device());
  ctx.ogates = ogates;
  ctx.log = log;
  bg::g_err.clear();
  return h->m->ProcessPackets(&ctx, ptrs.data(), cnt);
}

int bg_module_process(bg_module *h, const bg_ctx *ctx, uint8_t *const *heads,
                      size_t cnt, uint16_t *ogates) {
  return process(h, ctx, heads, nullptr, cnt, ogates, nullptr);
}

int bg_module_process_meta(bg_module *h, const bg_ctx *ctx, uint8_t *const *heads,
                           uint8_t *const *metas, size_t cnt, uint16_t *ogates) {
  return process(h, ctx, heads, metas, cnt, ogates, nullptr);
}

int bg_module_process_batches(bg_module *h, const bg_ctx *ctx,
                              uint8_t *const *heads, size_t cnt,
                              uint16_t *ogates, uint16_t *batch_gate,
                              uint32_t *batch_len, uint32_t *pkt_idx,
                              size_t *nbatches, size_t *ndead) {
  EmitLog log;
  int r = process(h, ctx, heads, nullptr, cnt, ogates, &log);
  if (r < 0) return r;
  size_t k = 0;
  for (size_t b = 0; b < log.batches.size(); b++) {
    batch_gate[b] = log.batches[b].gate;
    batch_len[b] = (uint32_t)log.batches[b].pkts.size();
    for (uint32_t i : log.batches[b].pkts) pkt_idx[k++] = i;
  }
  for (uint32_t i : log.dead) pkt_idx[k++] = i;
  *nbatches = log.batches.size();
  *ndead = log.dead.size();
  return 0;
}

// A worker's loop over this module with the synchronous drop-in path:
// ProcessBatch on each `burst` of packets in turn (Source -> module -> Sink).
int bg_module_run(bg_module *h, const bg_ctx *ctx, uint8_t *const *heads,
                  size_t n, size_t burst, uint16_t *ogates) {
  if (burst < 1) return fail(EINVAL, "burst must be >= 1");
  for (size_t i = 0; i < n; i += burst) {
    int r = process(h, ctx, heads + i, nullptr, std::min(burst, n - i), ogates + i, nullptr);
    if (r < 0) return r;
  }
  return 0;
}

int bg_module_connect(bg_module *h, uint16_t ogate, int connected) {
  if (ogate >= MAX_GATES) return fail(EINVAL, "ogate %hu not in [0,%d)", ogate, MAX_GATES);
  std::unique_lock<std::shared_mutex> lk(h->mu);
  h->m->ConnectOGate(ogate, connected != 0);
  return 0;
}

int bg_module_process_device(bg_module *h, const bg_ctx *ctx, void *d_frames,
                             size_t stride, size_t n, uint16_t *d_ogates,
                             bg_stream_t stream) {
  std::shared_lock<std::shared_mutex> lk(h->mu);
  const bg_ctx c = ResolveCtx(ctx, h->m->device());
  int r = bg::set_device(c.device);
  if (r) return r;
  return h->m->ProcessDevice(c, d_frames, stride, n, d_ogates, stream);
}

int bg_module_set_device(bg_module *h, int device) {
  int r = bg::set_device(device);
  if (r) return r;
  std::unique_lock<std::shared_mutex> lk(h->mu);
  h->m->set_device(device);
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
  std::unique_lock<std::shared_mutex> lk(h->mu);
  bg::g_err.clear();
  int r = h->m->BindMeta(meta_off, nm, off);
  if (r == -ENOTSUP && bg::g_err.empty())
    return fail(ENOTSUP, "'%s' has no metadata fields on its datapath",
                h->mclass.c_str());
  return r;
}

int bg_module_attr(const bg_module *h, int i, char *name, size_t cap, uint32_t *size) {
  const auto &a = h->m->all_attrs();
  if (i < 0 || (size_t)i >= a.size()) return 0;
  if (name && cap) snprintf(name, cap, "%s", a[(size_t)i].name.c_str());
  if (size) *size = (uint32_t)a[(size_t)i].size;
  return 1;
}

int bg_module_desc(const bg_module *h, char *buf, size_t len) {
  std::string d = h->m->GetDesc();
  if (buf && len) {
    snprintf(buf, len, "%s", d.c_str());
  }
  return (int)d.size();
}

}  // extern "C"
