// A minimal stand-in for bessd's core headers, exposing exactly the names
// the integration/bessd/*_gpu.cc plugin wrappers use, so that the wrappers
// compile and register here as they would inside bessd (tests only):
//
//   Module, Context, bess::Packet / PacketBatch       core/module.h, packet.h
//   Command / Commands, THREAD_SAFE / THREAD_UNSAFE   core/commands.h:54-72
//   MODULE_CMD_FUNC / MODULE_INIT_FUNC                core/module.h:82-102
//   CommandResponse, CommandSuccess / CommandFailure  core/message.h:44-53
//   EmitPacket / DropPacket                           core/module.h:534-594
//   ADD_MODULE -> ModuleBuilder::RegisterModuleClass  core/module.h:719-733
//   gate_idx_t, MAX_GATES, DROP_GATE, SNBUF_*         core/gate.h, snbuf_layout.h
//   RegisterTask / RunTask / task_result, is_task_,    core/module.h:198-311,
//   max_allowed_workers_, propagate_workers_           core/task.h:40-44
//   Worker::kMaxWorkers, current_worker.socket(),     core/worker.h:77,101,143,155
//   num_workers
//   bess::PacketPool (GetDefaultPool, Capacity, Size, core/packet_pool.h:32-64
//   AllocBulk), bess::Packet::Free                    core/packet.h:194-203
//
// EmitPacket keeps bessd's rule (module.h:546-549): an out-of-range or
// unconnected output gate drops the packet.
#ifndef BESSD_SHELL_MODULE_H_
#define BESSD_SHELL_MODULE_H_

#include <errno.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "pb/module_msg.pb.h"

typedef uint16_t gate_idx_t;
#define MAX_GATES 8192
#define DROP_GATE MAX_GATES

#define SNBUF_MBUF 128
#define SNBUF_IMMUTABLE 64
#define SNBUF_METADATA 128
#define SNBUF_SCRATCHPAD 64
#define SNBUF_HEADROOM 128
#define SNBUF_DATA 2048
#define SNBUF_METADATA_OFF (SNBUF_MBUF + SNBUF_IMMUTABLE)
#define SNBUF_HEADROOM_OFF (SNBUF_METADATA_OFF + SNBUF_METADATA + SNBUF_SCRATCHPAD)
#define SNBUF_SIZE (SNBUF_HEADROOM_OFF + SNBUF_HEADROOM + SNBUF_DATA)

class Worker {
 public:
  static const int kMaxWorkers = 64;  // core/worker.h:77
  int socket() const { return 0; }    // the shell: one socket
};
// core/worker.h:143,155: the calling worker; workers launched
inline thread_local Worker current_worker;
inline int num_workers = 1;

typedef uint16_t task_id_t;
#define INVALID_TASK_ID ((task_id_t)-1)

// core/task.h:40-44
struct task_result {
  bool block;
  uint32_t packets;
  uint64_t bits;
};

// The DPDK mempool surface a plugin uses to find the packet memory
// (rte_mempool.h, DPDK 19.11: rte_mempool_mem_iter over the pool's memory
// chunks): the shell's pool is one chunk.
struct rte_mempool {
  void *addr = nullptr;
  size_t len = 0;
};
struct rte_mempool_memhdr {
  void *addr;
  size_t len;
};
typedef void(rte_mempool_mem_cb_t)(struct rte_mempool *mp, void *opaque,
                                   struct rte_mempool_memhdr *memhdr, unsigned mem_idx);
inline uint32_t rte_mempool_mem_iter(struct rte_mempool *mp, rte_mempool_mem_cb_t *cb,
                                     void *arg) {
  if (!mp || !mp->addr) return 0;
  rte_mempool_memhdr h{mp->addr, mp->len};
  cb(mp, arg, &h, 0);
  return 1;
}

namespace bess {

class PacketPool;

// an snbuf: the packet object at the start of its slot, its data at
// SNBUF_HEADROOM_OFF + data_off
class Packet {
 public:
  template <typename T = void *>
  T head_data() {
    return reinterpret_cast<T>(reinterpret_cast<uint8_t *>(this) + SNBUF_HEADROOM_OFF +
                               data_off_);
  }
  // the metadata area (core/packet.h:100-104: Packet::metadata_, at
  // SNBUF_METADATA_OFF of the snbuf)
  template <typename T = void *>
  T metadata() {
    return reinterpret_cast<T>(reinterpret_cast<uint8_t *>(this) + SNBUF_METADATA_OFF);
  }
  uint16_t data_off() const { return data_off_; }
  void set_data_off(uint16_t v) { data_off_ = v; }
  uint32_t total_len() const { return total_len_; }
  void set_total_len(uint32_t v) { total_len_ = v; }
  uint16_t data_len() const { return data_len_; }
  void set_data_len(uint16_t v) { data_len_ = v; }
  // back to the packet's pool (a pool-less packet: the shell's static
  // buffers of the `frames` command) -- core/packet.h:194-203
  static inline void Free(Packet *p);
  static inline void Free(Packet **pkts, size_t cnt) {
    for (size_t i = 0; i < cnt; i++) Free(pkts[i]);
  }
  PacketPool *pool() const { return pool_; }
  void set_pool(PacketPool *p) { pool_ = p; }
  // the shell's pool position of the packet (its Sink's bookkeeping)
  uint32_t pool_index() const { return pool_index_; }
  void set_pool_index(uint32_t i) { pool_index_ = i; }

 private:
  uint16_t data_off_ = SNBUF_HEADROOM;
  uint16_t data_len_ = 0;
  uint32_t total_len_ = 0;
  uint32_t pool_index_ = 0;
  PacketPool *pool_ = nullptr;
};

// core/packet_pool.h: a fixed set of snbufs (mempool objects of SNBUF_SIZE +
// 64 bytes, the frame at +512), handed out and taken back by every worker;
// each thread keeps a cache of up to 512 (rte_mempool's per-lcore cache) and
// trades whole magazines of 256 with the shared list, so the lock is held for
// a pointer move, not while 256 pointers another core wrote are copied
class PacketPool {
 public:
  static const size_t kObj = SNBUF_SIZE + 64;
  static PacketPool *GetDefaultPool(int) { return default_pool(); }
  static PacketPool *&default_pool() {
    static PacketPool *p = nullptr;
    return p;
  }
  explicit PacketPool(size_t capacity) : capacity_(capacity) {
    // (page-aligned: the memory a plugin registers for device access)
    mem_ = static_cast<uint8_t *>(aligned_alloc(4096, (capacity * kObj + 4095) / 4096 * 4096));
    memset(mem_, 0, capacity * kObj);
    mp_.addr = mem_;
    mp_.len = capacity * kObj;
    std::vector<Packet *> m;
    for (size_t i = capacity; i-- > 0;) {
      Packet *p = new (mem_ + i * kObj) Packet();
      p->set_pool(this);
      m.push_back(p);
      if (m.size() == kMag || i == 0) {
        avail_ += m.size();
        mags_.push_back(std::move(m));
        m.clear();
      }
    }
    gen_ = ++generation();
  }
  ~PacketPool() {
    ++generation();  // thread caches of this pool are stale now
    free(mem_);
  }
  size_t Capacity() const { return capacity_; }
  rte_mempool *pool() { return &mp_; }  // packet_pool.h:67
  size_t Size() const {  // available: the shared list (thread caches not counted)
    std::lock_guard<std::mutex> lk(mu_);
    return avail_;
  }
  // all or nothing (packet_pool.h:56-58)
  bool AllocBulk(Packet **pkts, size_t count, size_t len = 0) {
    Cache &c = cache();
    while (c.v.size() < count) {
      std::vector<Packet *> m;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (mags_.empty()) break;
        m = std::move(mags_.back());
        mags_.pop_back();
        avail_ -= m.size();
      }
      c.v.insert(c.v.end(), m.begin(), m.end());
    }
    if (c.v.size() < count) return false;
    for (size_t i = 0; i < count; i++) {
      pkts[i] = c.v.back();
      c.v.pop_back();
      pkts[i]->set_data_off(SNBUF_HEADROOM);
      pkts[i]->set_data_len((uint16_t)len);
      pkts[i]->set_total_len((uint32_t)len);
    }
    return true;
  }
  void Put(Packet *p) {
    Cache &c = cache();
    c.v.push_back(p);
    if (c.v.size() >= kCache) Spill(c, kMag);
  }
  // a worker thread's cache back into the shared list (thread exit)
  void FlushThreadCache() {
    Cache &c = cache();
    Spill(c, c.v.size());
  }

 private:
  static const size_t kCache = 512;
  static const size_t kMag = 256;
  struct Cache {
    uint64_t gen = 0;
    PacketPool *owner = nullptr;
    std::vector<Packet *> v;
    ~Cache() {
      if (owner && gen == generation()) owner->Spill(*this, v.size());
    }
  };
  static std::atomic<uint64_t> &generation() {
    static std::atomic<uint64_t> g{0};
    return g;
  }
  Cache &cache() {
    thread_local Cache c;
    if (c.owner != this || c.gen != gen_) {
      c.owner = this;
      c.gen = gen_;
      c.v.clear();
    }
    return c;
  }
  void Spill(Cache &c, size_t n) {
    n = std::min(n, c.v.size());
    if (!n) return;
    std::vector<Packet *> m(c.v.end() - (std::ptrdiff_t)n, c.v.end());
    c.v.resize(c.v.size() - n);
    std::lock_guard<std::mutex> lk(mu_);
    avail_ += m.size();
    mags_.push_back(std::move(m));
  }
  size_t capacity_;
  uint8_t *mem_ = nullptr;
  rte_mempool mp_;
  uint64_t gen_ = 0;
  mutable std::mutex mu_;
  std::vector<std::vector<Packet *>> mags_;  // magazines of <= kMag
  size_t avail_ = 0;
};

inline void Packet::Free(Packet *p) {
  if (p->pool_) p->pool_->Put(p);
}

class PacketBatch {
 public:
  static const size_t kMaxBurst = 32;
  int cnt() const { return cnt_; }
  Packet **pkts() { return pkts_; }
  void clear() { cnt_ = 0; }
  void add(Packet *p) { pkts_[cnt_++] = p; }

 private:
  int cnt_ = 0;
  Packet *pkts_[kMaxBurst];
};

namespace metadata {
// core/metadata.h: an attribute's access mode; the offset of an attribute
// no upstream module writes (kMetadataOffsetNoRead)
struct Attribute {
  enum class AccessMode { kRead = 0, kWrite, kUpdate };
  std::string name;
  size_t size;
  AccessMode mode;
};
typedef int16_t mt_offset_t;
static const mt_offset_t kMetadataOffsetNoRead = -2;
}  // namespace metadata

}  // namespace bess

struct Context {
  uint64_t current_tsc = 0;
  uint64_t current_ns = 0;
  int wid = 0;
  gate_idx_t current_igate = 0;
  // where each packet went (the shell's stand-in for the task's batches)
  std::vector<std::pair<bess::Packet *, gate_idx_t>> emitted;
  std::vector<bess::Packet *> dropped;
  // (verify) emission order: a number from one counter shared by all
  // workers, per packet (Packet::pool_index), taken when EmitPacket runs
  std::atomic<uint64_t> *emit_counter = nullptr;
  std::vector<uint64_t> *emit_seq = nullptr;
};

class CommandResponse {
 public:
  bool has_error() const { return code_ != 0; }
  int code() const { return code_; }
  const std::string &errmsg() const { return msg_; }
  const std::string &data() const { return data_; }
  void set_error(int c, const std::string &m) {
    code_ = c;
    msg_ = m;
  }
  void set_data(const std::string &d) { data_ = d; }

 private:
  int code_ = 0;
  std::string msg_, data_;
};

inline CommandResponse CommandSuccess() { return CommandResponse(); }
inline CommandResponse CommandSuccess(const google::protobuf::Message &m) {
  CommandResponse r;
  r.set_data(m.SerializeAsString());
  return r;
}
inline CommandResponse CommandFailure(int code, const char *fmt = nullptr, ...) {
  CommandResponse r;
  char b[512] = "";
  if (fmt) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof(b), fmt, ap);
    va_end(ap);
  }
  r.set_error(code, b);
  return r;
}

class Module;
using module_cmd_func_t =
    std::function<CommandResponse(Module *, const google::protobuf::Any &)>;

struct Command {
  enum ThreadSafety { THREAD_UNSAFE = 0, THREAD_SAFE = 1 };
  std::string cmd;
  std::string arg_type;
  module_cmd_func_t func;
  ThreadSafety mt_safe;
};
using Commands = std::vector<Command>;

template <typename T, typename M>
static inline module_cmd_func_t MODULE_CMD_FUNC(CommandResponse (M::*fn)(const T &)) {
  return [fn](Module *m, const google::protobuf::Any &arg) {
    T a;
    arg.UnpackTo(&a);
    return (static_cast<M *>(m)->*fn)(a);
  };
}
#define MODULE_INIT_FUNC MODULE_CMD_FUNC

class Module {
 public:
  static const gate_idx_t kNumIGates = 1;
  static const gate_idx_t kNumOGates = 1;
  static const Commands cmds;

  virtual ~Module() = default;
  // modules without an Init of their own (e.g. UpdateTTL) take EmptyArg
  CommandResponse Init(const bess::pb::EmptyArg &) { return CommandSuccess(); }
  virtual void DeInit() {}
  virtual void ProcessBatch(Context *, bess::PacketBatch *) {}
  virtual struct task_result RunTask(Context *, bess::PacketBatch *, void *) {
    return {.block = true, .packets = 0, .bits = 0};
  }
  virtual std::string GetDesc() const { return ""; }

  // Module::RegisterTask (core/module.cc:156-167): the shell's scheduler
  // runs each registered task from the worker it is given to
  task_id_t RegisterTask(void *arg) {
    tasks_.push_back(arg);
    return (task_id_t)(tasks_.size() - 1);
  }
  size_t num_tasks() const { return tasks_.size(); }
  bool is_task() const { return is_task_ || !tasks_.empty(); }
  int max_allowed_workers() const { return max_allowed_workers_; }

  // ConnectModules: the output gates with a next module
  void ConnectOGate(gate_idx_t g) {
    if (g >= ogates_.size()) ogates_.resize((size_t)g + 1, false);
    ogates_[g] = true;
  }
  void EmitPacket(Context *ctx, bess::Packet *pkt, gate_idx_t ogate = 0) {
    if (ogates_.size() <= ogate || !ogates_[ogate]) {  // module.h:546-549
      DropPacket(ctx, pkt);
      return;
    }
    ctx->emitted.push_back({pkt, ogate});
    if (ctx->emit_seq) (*ctx->emit_seq)[pkt->pool_index()] = (*ctx->emit_counter)++;
  }
  void DropPacket(Context *ctx, bess::Packet *pkt) { ctx->dropped.push_back(pkt); }
  // core/module.h:530-532: the whole batch to output gate 0
  void RunNextModule(Context *ctx, bess::PacketBatch *batch) {
    for (int i = 0; i < batch->cnt(); i++) EmitPacket(ctx, batch->pkts()[i], 0);
  }

  // Module::AddMetadataAttr / attr_offset (core/module.h:294-328): the
  // shell's pipeline packs the attributes in registration order (bessd's
  // allocator, core/metadata.cc, places them by its own rules; a script may
  // place them with set_attr_offset, as Pipeline::ComputeMetadataOffsets
  // does before the workers resume)
  int AddMetadataAttr(const std::string &name, size_t size,
                      bess::metadata::Attribute::AccessMode mode) {
    for (const auto &a : attrs_)
      if (a.name == name) return -EEXIST;
    int32_t off = 0;
    for (const auto &a : attrs_) off += (int32_t)a.size;
    attrs_.push_back(bess::metadata::Attribute{name, size, mode});
    attr_offsets_.push_back(off);
    return (int)attrs_.size() - 1;
  }
  bess::metadata::mt_offset_t attr_offset(size_t attr_id) const {
    return (bess::metadata::mt_offset_t)attr_offsets_[attr_id];
  }
  void set_attr_offset(size_t attr_id, bess::metadata::mt_offset_t off) {
    if (attr_id < attr_offsets_.size()) attr_offsets_[attr_id] = off;
  }
  size_t num_attrs() const { return attrs_.size(); }
  const std::vector<bess::metadata::Attribute> &all_attrs() const { return attrs_; }

 protected:
  bool is_task_ = false;            // core/module.h:464
  int max_allowed_workers_ = 1;     // core/module.h:485 (default 1)
  bool propagate_workers_ = true;   // core/module.h:491

 private:
  std::vector<void *> tasks_;
  std::vector<bool> ogates_;
  std::vector<bess::metadata::Attribute> attrs_;
  std::vector<int32_t> attr_offsets_;
};
inline const Commands Module::cmds = {};

// ModuleBuilder::RegisterModuleClass (core/module.h:108-172): what bessd
// records per class, kept for inspection
struct ModuleClass {
  std::function<Module *()> make;
  std::string name_template, help;
  gate_idx_t igates, ogates;
  Commands cmds;
  module_cmd_func_t init;
};
inline std::map<std::string, ModuleClass> &module_classes() {
  static std::map<std::string, ModuleClass> m;
  return m;
}
struct ModuleBuilder {
  static bool RegisterModuleClass(std::function<Module *()> make, const std::string &cls,
                                  const std::string &tmpl, const std::string &help,
                                  gate_idx_t ig, gate_idx_t og, const Commands &cmds,
                                  module_cmd_func_t init) {
    return module_classes()
        .emplace(cls, ModuleClass{make, tmpl, help, ig, og, cmds, init})
        .second;
  }
  static bool DeregisterModuleClass(const std::string &cls) {
    return module_classes().erase(cls) > 0;
  }
};

#define DEF_MODULE(_MOD, _NAME_TEMPLATE, _HELP)                                        \
  class _MOD##_class {                                                                 \
   public:                                                                             \
    _MOD##_class() {                                                                   \
      ModuleBuilder::RegisterModuleClass([]() -> Module * { return new _MOD(); }, #_MOD, \
                                         _NAME_TEMPLATE, _HELP, _MOD::kNumIGates,      \
                                         _MOD::kNumOGates, _MOD::cmds,                 \
                                         MODULE_INIT_FUNC(&_MOD::Init));               \
    }                                                                                  \
    ~_MOD##_class() { ModuleBuilder::DeregisterModuleClass(#_MOD); }                   \
  };

#define ADD_MODULE(_MOD, _NAME_TEMPLATE, _HELP) \
  DEF_MODULE(_MOD, _NAME_TEMPLATE, _HELP);      \
  static _MOD##_class _MOD##_singleton;

#endif  // BESSD_SHELL_MODULE_H_
