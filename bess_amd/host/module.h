// module.h -- the slice of BESS's module API that the classification
// modules use, so they keep the reference's surface:
//
//   Module::ProcessBatch(Context *, bess::PacketBatch *)  core/module.h:226
//   EmitPacket / DropPacket                               core/module.h:534-594
//   CommandResponse, CommandSuccess / CommandFailure      core/message.h:44-53
//   Commands {cmd, arg_type, func, THREAD_SAFE|UNSAFE}    core/commands.h:57-72
//   ADD_MODULE registration (first registration wins)     core/module.h:719-733
//   gate_idx_t / MAX_GATES / DROP_GATE                    core/gate.h:49-58
//
// In a bessd build the same module sources would include the real headers;
// this file is the stand-alone host shell used here (no DPDK / protobuf /
// gRPC in the image). Packets are plain head pointers into frame buffers.
#ifndef BESS_AMD_HOST_MODULE_H_
#define BESS_AMD_HOST_MODULE_H_

#include <errno.h>
#include <stdarg.h>
#include <stdint.h>

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "pb.h"

typedef uint16_t gate_idx_t;
#define MAX_GATES 8192
#define DROP_GATE MAX_GATES
#define INVALID_GATE UINT16_MAX

namespace bess {

// A packet as the classifiers see it: Packet::head_data() (core/packet.h:
// 84-94) plus the bytes that may be read/written from there.
class Packet {
 public:
  Packet() = default;
  Packet(uint8_t *head, uint32_t span, uint32_t index, uint8_t *meta = nullptr)
      : head_(head), meta_(meta), span_(span), index_(index) {}
  template <typename T = void *>
  T head_data() const {
    return reinterpret_cast<T>(head_);
  }
  // the packet's metadata area (Packet::metadata(), core/packet.h; the
  // snbuf's SNBUF_METADATA bytes), when the caller passed it
  template <typename T = void *>
  T metadata() const {
    return reinterpret_cast<T>(meta_);
  }
  uint32_t span() const { return span_; }
  uint32_t index() const { return index_; }

 private:
  uint8_t *head_ = nullptr;
  uint8_t *meta_ = nullptr;
  uint32_t span_ = 0;
  uint32_t index_ = 0;
};

// core/pktbatch.h:40-75
class PacketBatch {
 public:
  static const size_t kMaxBurst = 32;
  int cnt() const { return cnt_; }
  Packet *const *pkts() const { return pkts_; }
  Packet **pkts() { return pkts_; }
  void clear() { cnt_ = 0; }
  void add(Packet *p) { pkts_[cnt_++] = p; }

 private:
  int cnt_ = 0;
  Packet *pkts_[kMaxBurst];
};

}  // namespace bess

// The batches a Task would run after one ProcessBatch call: EmitPacket
// appends each packet to its output gate's batch and starts a new batch
// when that one holds kMaxBurst packets (core/module.h:543-594; the igate
// batches go onto the task's run list in the order they were started,
// Task::AddToRun); DropPacket collects the dead batch (534-541).
struct EmitLog {
  struct Batch {
    gate_idx_t gate;
    std::vector<uint32_t> pkts;  // Packet::index() of each packet, in order
  };
  std::vector<Batch> batches;    // AddToRun order
  std::vector<uint32_t> dead;    // dropped packets, in drop order
  std::map<gate_idx_t, size_t> open;  // gate -> its batch being filled
};

// Per-call context (core/module.h:59-75): the batch's input gate, the
// worker's clock and the device of this call (bg_ctx: never module state),
// and where each packet went.
struct Context {
  bg_ctx call{};               // current_igate, current_ns, device, wid
  uint16_t *ogates = nullptr;  // indexed by Packet::index(); DROP_GATE: dropped
  EmitLog *log = nullptr;      // optional: the gate batches
  uint64_t deadends = 0;       // deadends_[ctx->wid] (module.h:455)
};

// bg_ctx with its defaults filled in (NULL: igate 0, the monotonic clock
// now; device -1: module_device)
bg_ctx ResolveCtx(const bg_ctx *c, int module_device);

class CommandResponse {
 public:
  int code() const { return code_; }
  const std::string &errmsg() const { return msg_; }
  const std::string &data() const { return data_; }
  void set_error(int code, const std::string &msg) {
    code_ = code;
    msg_ = msg;
  }
  void set_data(const std::string &d) { data_ = d; }

 private:
  int code_ = 0;
  std::string msg_;
  std::string data_;  // serialized response message
};

CommandResponse CommandSuccess();
CommandResponse CommandSuccess(const bess::pb::Message &m);
CommandResponse CommandFailure(int code, const char *fmt = nullptr, ...)
    __attribute__((format(printf, 2, 3)));

class Module;

// The staged row of one packet (bg_pipe slots, Module::ProcessPackets):
// frame bytes [lo, hi) at row offset 0, then, for a module whose attr_name
// fields read the metadata area (Module::MetaWindow [mlo, mhi)), those
// metadata bytes at row offset StagedMetaAt(lo, hi) -- so metadata byte 0
// sits at row offset StagedMetaAt(lo, hi) - mlo (bg_em_classify_staged's
// meta_row). Row stride: StagedStride.
// (at least 16: a module whose fields are all attributes stages one chunk
// of frame bytes, as the pipe and the host path stage [lo, max(hi, lo + 1)))
inline int StagedMetaAt(int lo, int hi) { return hi > lo ? (hi - lo + 15) / 16 * 16 : 16; }
inline size_t StagedStride(int lo, int hi, int mlo, int mhi) {
  return (size_t)StagedMetaAt(lo, hi) + (size_t)((mhi - mlo + 15) / 16 * 16);
}

// A persistent ring (bg_ring) serving a module's staged windows on one
// device, shared by the module's pipes (each on a lane of its own while
// there are lanes) and by their in-flight slots: it is destroyed -- its
// grid stopped -- when the last of them lets go, so a rule change retires
// it only once every slot submitted under the old rules has finished.
struct PipeRing {
  bg_ring *r = nullptr;
  int device = 0;
  int lanes = 0;
  uint64_t version = 0;  // the rules it classifies with
  int meta_row = 0;      // where its rows carry the metadata (StagedMetaAt)
  std::atomic<int> next_lane{0};
  // pipes past `lanes` share a lane; bg_ring's lanes take one thread at a
  // time (EBUSY otherwise), so a pipe holds its lane's lock around each call
  std::unique_ptr<std::mutex[]> lane_mu;
  ~PipeRing() { bg_ring_destroy(r); }
};

struct Command {
  enum ThreadSafety { THREAD_UNSAFE = 0, THREAD_SAFE = 1 };
  std::string cmd;
  std::string arg_type;
  std::function<CommandResponse(Module *, const void *, size_t)> func;
  ThreadSafety mt_safe;
};
using Commands = std::vector<Command>;

// MODULE_CMD_FUNC: adapt `CommandResponse C::f(const Arg &)` to the
// serialized-argument form the control plane delivers.
template <typename C, typename Arg>
std::function<CommandResponse(Module *, const void *, size_t)> ModuleCmdFunc(
    CommandResponse (C::*f)(const Arg &)) {
  return [f](Module *m, const void *arg, size_t len) {
    Arg a;
    if (!a.ParseFromArray(arg, len))
      return CommandFailure(EINVAL, "failed to parse argument");
    return (static_cast<C *>(m)->*f)(a);
  };
}
#define MODULE_CMD_FUNC(f) ModuleCmdFunc(f)

class Module {
 public:
  virtual ~Module() = default;
  // core/module.h:226: every module runs its batch on the device through
  // ProcessPackets
  virtual void ProcessBatch(Context *ctx, bess::PacketBatch *batch) {
    ProcessPackets(ctx, batch->pkts(), (size_t)batch->cnt());
  }
  // Any number of packets in one synchronous call (BESS hands ProcessBatch
  // <= 32): the DeviceWindow bytes of each packet are staged in the calling
  // thread's pinned buffers, ProcessDeviceWindow runs on the thread's own
  // stream, the gates (and, for writing modules, the header lines) come
  // back, then each packet is emitted on its gate (BG_GATE_NONE: not
  // emitted). Re-entrant: many workers may run it on one module at once
  // (module.cc). Returns 0 or -errno (every packet dropped).
  virtual int ProcessPackets(Context *ctx, bess::Packet *const *pkts,
                             size_t cnt);
  virtual std::string GetDesc() const { return ""; }
  virtual const Commands &cmds() const = 0;
  // Device-resident datapath over a frame slab (libbessgpu.so) for one
  // call's context: c.device is resolved (>= 0) and is the calling thread's
  // current HIP device; c.igate / c.now_ns are the batch's.
  virtual int ProcessDevice(const bg_ctx &c, void *d_frames, size_t stride,
                            size_t n, uint16_t *d_ogates, void *stream) = 0;
  // Which context fields the device datapath reads (a bg_pipe slot holds
  // packets of one value of them).
  enum : unsigned { kCtxIgate = 1, kCtxNow = 2 };
  virtual unsigned CtxUse() const { return 0; }
  // Host ingress/egress staging (bg_pipe, bess_amd/host/pipe.cc): the frame
  // bytes [*lo, *hi) the device datapath reads, and whether it writes frame
  // bytes that must go back into the packet buffers.
  virtual void DeviceWindow(int *lo, int *hi, bool *writeback) const {
    *lo = 0;
    *hi = 2048;  // SNBUF_DATA (core/snbuf_layout.h:34-68)
    *writeback = false;
  }
  // How many bytes from the head a writeback datapath reads of a frame whose
  // data_len is `len` (the pipe stages that many, capped to the window, and
  // zero-pads only past them). The reference's checksum modules sum the
  // byte counts the headers give, whatever data_len is: they
  // override this.
  virtual size_t StageReach(const uint8_t *frame, size_t len) const {
    (void)frame;
    return len;
  }
  // ProcessDevice over frames by pointer (d_ptrs[i]: the device address of
  // packet i's head in host-registered memory, `span` bytes each; the
  // module writes in place): the zero-copy slots of a writeback pipe.
  // -ENOTSUP: the module has no such datapath (n == 0 asks).
  virtual int ProcessDevicePtrs(const bg_ctx &c, const uint64_t *d_ptrs, size_t span,
                                size_t n, uint16_t *d_ogates, void *stream) {
    (void)c;
    (void)d_ptrs;
    (void)span;
    (void)n;
    (void)d_ogates;
    (void)stream;
    return -ENOTSUP;
  }
  // The metadata bytes [*mlo, *mhi) the device datapath reads (attr_name
  // fields), staged after the frame window (StagedMetaAt);
  // none: *mlo == *mhi. -errno while the attribute offsets are unbound.
  virtual int MetaWindow(int *mlo, int *mhi) const {
    *mlo = *mhi = 0;
    return 0;
  }
  // ProcessDevice over staged rows: byte 0 of row i is frame offset
  // `win_off` of packet i (= DeviceWindow's lo), followed by the packet's
  // metadata bytes as StagedMetaAt lays them out when MetaWindow has any.
  virtual int ProcessDeviceWindow(const bg_ctx &c, void *d_win, size_t wstride,
                                  size_t n, int win_off, uint16_t *d_ogates,
                                  void *stream) {
    if (win_off != 0) return -EINVAL;
    return ProcessDevice(c, d_win, wstride, n, d_ogates, stream);
  }
  // The ring a pipe submits its slots to on `device` (their windows start at
  // DeviceWindow's lo), with the gate of packets no rule matches; null when
  // the module has none (the pipe launches H2D/kernel/D2H per slot). A
  // module returns a new ring once its rules changed (<0: -errno).
  virtual int PipeRingFor(int device, std::shared_ptr<PipeRing> *out, uint16_t *dflt) {
    (void)device;
    (void)dflt;
    out->reset();
    return 0;
  }
  // Whether `ring` (from PipeRingFor) is still the one PipeRingFor would
  // return -- same rules, same row layout -- with the current default gate:
  // the per-slot check without PipeRingFor's lock (workers share it).
  virtual bool PipeRingCurrent(const PipeRing &ring, uint16_t *dflt) const {
    (void)ring;
    (void)dflt;
    return false;
  }
  // attr_name fields: metadata area at slot offset meta_off (-1: none, the
  // attribute offsets only -- staged rows carry the metadata bytes),
  // attribute offsets by name (bg_module_bind_meta). Modules without attr
  // fields on their datapath: ENOTSUP.
  virtual int BindMeta(int meta_off, const std::vector<std::string> &names,
                       const std::vector<int32_t> &offsets) {
    (void)meta_off;
    (void)names;
    (void)offsets;
    return -ENOTSUP;
  }
  // offsets of this module's attributes (by id) from a name -> offset list;
  // -1 for names not given
  std::vector<int32_t> AttrOffsets(const std::vector<std::string> &names,
                                   const std::vector<int32_t> &offsets) const {
    std::vector<int32_t> r(attrs_.size(), -1);
    for (size_t i = 0; i < attrs_.size(); i++)
      for (size_t j = 0; j < names.size(); j++)
        if (names[j] == attrs_[i].name) r[i] = offsets[j];
    return r;
  }
  // the device of calls whose bg_ctx says -1 (control path)
  void set_device(int d) { device_ = d; }
  int device() const { return device_; }

  // Module::AddMetadataAttr (core/module.cc:248-285): per-module metadata
  // attributes; returns the attribute id or -errno.
  struct Attribute {
    std::string name;
    size_t size;
  };
  int AddMetadataAttr(const std::string &name, size_t size) {
    if (attrs_.size() >= 16) return -ENOSPC;         // kMaxAttrsPerModule
    if (name.empty()) return -EINVAL;
    if (size < 1 || size > 32) return -EINVAL;       // kMetadataAttrMaxSize
    for (const auto &a : attrs_)
      if (a.name == name) return -EEXIST;
    attrs_.push_back(Attribute{name, size});
    return (int)attrs_.size() - 1;
  }
  const std::vector<Attribute> &all_attrs() const { return attrs_; }

  // Output gates the pipeline connected (ConnectModules). Until the first
  // ConnectOGate every gate < MAX_GATES counts as connected.
  void ConnectOGate(gate_idx_t g, bool on) {
    if (!explicit_ogates_) {
      ogates_.clear();
      explicit_ogates_ = true;
    }
    if (g >= ogates_.size()) ogates_.resize((size_t)g + 1, false);
    ogates_[g] = on;
  }
  bool OGateConnected(gate_idx_t g) const {
    if (!explicit_ogates_) return g < MAX_GATES;
    return g < ogates_.size() && ogates_[g];
  }

  // core/module.h:543-594: a gate that is out of range or not connected
  // drops the packet (546-549); otherwise the packet joins the gate's batch.
  void EmitPacket(Context *ctx, bess::Packet *pkt, gate_idx_t ogate) {
    if (!OGateConnected(ogate)) {
      DropPacket(ctx, pkt);
      return;
    }
    ctx->ogates[pkt->index()] = ogate;
    if (EmitLog *l = ctx->log) {
      auto it = l->open.find(ogate);
      if (it == l->open.end() ||
          l->batches[it->second].pkts.size() >= bess::PacketBatch::kMaxBurst) {
        l->batches.push_back(EmitLog::Batch{ogate, {}});
        l->open[ogate] = l->batches.size() - 1;
        it = l->open.find(ogate);
      }
      l->batches[it->second].pkts.push_back(pkt->index());
    }
  }
  // core/module.h:534-541
  void DropPacket(Context *ctx, bess::Packet *pkt) {
    ctx->ogates[pkt->index()] = DROP_GATE;
    ctx->deadends++;
    if (ctx->log) ctx->log->dead.push_back(pkt->index());
  }

 protected:
  int device_ = 0;
  std::vector<Attribute> attrs_;
  std::vector<bool> ogates_;
  bool explicit_ogates_ = false;
};

// ModuleBuilder (core/module.h:108-172): class name -> factory taking the
// serialized <Class>Arg and running Init.
class ModuleBuilder {
 public:
  using Factory = std::function<CommandResponse(const void *, size_t,
                                                std::unique_ptr<Module> *)>;
  static bool RegisterModuleClass(const std::string &class_name,
                                  const std::string &name_template,
                                  const std::string &help, Factory f);
  static const ModuleBuilder *Find(const std::string &class_name);
  static std::vector<std::string> Classes();
  const std::string &name_template() const { return name_template_; }
  const std::string &help() const { return help_; }
  CommandResponse Create(const void *arg, size_t len,
                         std::unique_ptr<Module> *out) const {
    return factory_(arg, len, out);
  }

 private:
  std::string name_template_, help_;
  Factory factory_;
};

template <typename C, typename Arg>
ModuleBuilder::Factory MakeFactory() {
  return [](const void *arg, size_t len, std::unique_ptr<Module> *out) {
    Arg a;
    if (!a.ParseFromArray(arg, len))
      return CommandFailure(EINVAL, "failed to parse %s argument", "module");
    std::unique_ptr<C> m(new C());
    CommandResponse r = m->Init(a);
    if (r.code() == 0) *out = std::move(m);
    return r;
  };
}

// ADD_MODULE(class, name_template, help) with the Init argument type.
#define ADD_MODULE_ARG(_MOD, _ARG, _NAME_TEMPLATE, _HELP)                     \
  static bool __module__##_MOD = ModuleBuilder::RegisterModuleClass(          \
      #_MOD, _NAME_TEMPLATE, _HELP, MakeFactory<_MOD, _ARG>());

struct bg_pipe;

// The C ABI's module handle (include/bessgpu.h bg_module_*).
struct bg_module {
  std::unique_ptr<Module> m;
  std::string mclass;
  // ProcessBatch calls, pipe launches and THREAD_SAFE commands share it;
  // THREAD_UNSAFE commands (which bessd runs only with workers paused,
  // core/module.cc:97-101) take it exclusively
  std::shared_mutex mu;
  // the pipes feeding this module: a THREAD_UNSAFE command first launches
  // their partly filled slots, so every packet submitted before a rule
  // change is classified with the rules it was submitted under
  std::mutex pipes_mu;
  std::set<bg_pipe *> pipes;
  // the owner's handle (bg_module_destroy) and every open pipe hold one
  // reference: a module destroyed under open pipes lives until the last
  // pipe goes (a host may tear its graph down in any order)
  std::atomic<int> refs{1};
};

// drop one reference (the owner's or a pipe's); the last one frees it
void ModuleUnref(bg_module *m);

// pipe.cc: launch a pipe's partly filled slot (its module's lock is held
// by the caller)
int PipeFlushLocked(bg_pipe *p);

#endif  // BESS_AMD_HOST_MODULE_H_
