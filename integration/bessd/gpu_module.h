// gpu_module.h -- the part every libbessgpu.so-backed bessd module shares.
//
// Drop these files into bessd's core/modules/ (they include "../module.h"
// and "../pb/module_msg.pb.h" like the built-in modules) and link the
// plugin with -lbessgpu. Each *_gpu.cc declares the same class name,
// gates, commands table and Init argument as the module it replaces, and
// forwards everything to the C ABI (include/bessgpu.h):
//   Init          -> bg_module_create(<class>, <Class>Arg bytes)
//   a command     -> bg_module_command(name, arg bytes) (+ response)
//   GetDesc       -> bg_module_desc
//   ProcessBatch  -> one of two datapaths:
//     deferred (CreateDeferred, the classifiers and checksum modules): the
//       Queue module's split (core/modules/queue.cc:173 ProcessBatch
//       enqueues, :190 RunTask emits; Init registers the task, :99-102).
//       Each worker (ctx->wid) has its own bg_pipe; ProcessBatch submits
//       the batch with its Packet* as cookies and the call's bg_ctx, then
//       emits what earlier batches have finished; the module's task
//       flushes a pipe whose worker went quiet and emits the rest. Packets
//       stay owned by the module until emitted or dropped (core/module.h:
//       224-226) and leave in submission order, so the per-gate order
//       within a batch is kept (module.h:268-272). Checksum modules' new
//       header lines are in the packet before it is emitted.
//     synchronous (Create): bg_module_process per batch (NAT, whose mapping
//       state is sequential and which allows one worker, nat.h).
// Gates map back onto bessd's EmitPacket / DropPacket, whose own check
// drops a packet sent to an out-of-range or unconnected gate
// (core/module.h:546-549).
#ifndef BESS_MODULES_GPU_MODULE_H_
#define BESS_MODULES_GPU_MODULE_H_

#include <algorithm>
#include <atomic>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../module.h"
#include "../pb/module_msg.pb.h"
#include "bessgpu.h"

class GpuModule : public Module {
 private:
  // one cache line per worker: its ProcessBatch calls count submits here
  struct alignas(64) Lane {
    std::atomic<bg_pipe *> pipe{nullptr};
    std::atomic<uint64_t> submits{0};  // ProcessBatch calls so far
    uint64_t seen = 0;                 // submits at the task's last visit
    std::atomic<bool> in_call{false};   // the owner is in ProcessBatch
    std::atomic<bool> draining{false};  // the task is emitting this pipe
    int win_lo = 0;                     // first data byte the pipe gathers
  };

 public:
  // the deferred datapath's pipes: packets per device launch, launches in
  // flight per worker, at most. A module served by a persistent ring
  // (ExactMatch, WildcardMatch) submits small slots at no launch cost
  // (8 x 1024; WildcardMatch 8 x 512, wildcard_match_gpu.cc); the
  // others launch H2D/kernel/D2H per slot and amortise that over up to 64 K
  // packets. Either way a worker's pipe holds no more than PipeBudget().
  static const size_t kPipeBatch = 65536;
  static const int kPipeDepth = 4;
  static const size_t kRingPipeBatch = 1024;
  static const int kRingPipeDepth = 8;

  // The packets one worker's pipe of a module may hold: a quarter of that
  // worker's share of its socket's packet pool (bessd allocates --buffers,
  // 262,144 per socket, core/opts.cc:127, for every port, module and worker
  // there), so deferred modules never starve the Sources. A full pipe
  // blocks the worker's submit until its oldest slot completes -- the
  // Queue module's backpressure (queue.cc:173-190), never a drop.
  static size_t PipeBudget() {
    size_t cap = 262144;
    if (bess::PacketPool *pool = bess::PacketPool::GetDefaultPool(current_worker.socket()))
      cap = pool->Capacity();
    const size_t w = num_workers > 0 ? (size_t)num_workers : 1;
    return std::max<size_t>(cap / (4 * w), 256);
  }

  void DeInit() override {
    for (Lane &l : lanes_) {
      bg_pipe *p = l.pipe.exchange(nullptr);
      if (!p) continue;
      // what is still queued is freed unemitted, as Queue::DeInit does
      (void)bg_pipe_flush(p);
      void *ck[256];
      long k;
      while ((k = bg_pipe_poll(p, 1, ck, nullptr, 256)) > 0)
        for (long i = 0; i < k; i++) bess::Packet::Free(static_cast<bess::Packet *>(ck[i]));
      bg_pipe_destroy(p);
    }
    for (void *base : registered_) PoolRegion(base, 0, -1);
    registered_.clear();
    bg_module_destroy(m_);
    m_ = nullptr;
  }

  // The module's task (deferred datapath): a worker's pipe that received
  // nothing since the last visit is flushed (its partly filled slot is
  // launched) and its finished packets leave (`packets`: those it handed
  // on, emitted, dropped or not emitted). A worker that keeps calling
  // ProcessBatch drains its own pipe there, so the task's worker never
  // carries the others' emissions; and a pipe's packets are emitted by one
  // thread at a time (the owner waits while the task empties its pipe), so
  // they leave in submission order.
  struct task_result RunTask(Context *ctx, bess::PacketBatch *, void *) override {
    uint32_t done = 0;
    std::shared_lock<std::shared_mutex> meta(meta_mu_, std::defer_lock);
    if (has_attrs_ && !meta.try_lock())  // a worker is re-binding the attributes
      return {.block = true, .packets = 0, .bits = 0};
    for (Lane &l : lanes_) {
      bg_pipe *p = l.pipe.load(std::memory_order_acquire);
      if (!p || bg_pipe_pending(p) == 0) continue;
      const uint64_t sub = l.submits.load(std::memory_order_relaxed);
      if (sub != l.seen) {
        l.seen = sub;
        continue;
      }
      if (l.draining.exchange(true)) continue;
      if (!l.in_call.load()) {  // (seq_cst: pairs with Enqueue's entry)
        (void)bg_pipe_flush(p);
        done += Drain(ctx, p);
      }
      l.draining.store(false, std::memory_order_release);
    }
    return {.block = done == 0, .packets = done, .bits = 0};
  }

  // The socket's packet pool registered for device access in place
  // (bg_host_register over the mempool's memory chunks, once per chunk and
  // process, counted per module): a checksum module's pipes then hand the
  // device each packet's head pointer, and the kernel reads the frame over
  // PCIe and writes the checksum words into the buffer -- no staging copy
  // (bg_pipe's zero-copy slots). Packets from elsewhere are staged as before.
  void UsePacketPoolInPlace() { in_place_ = true; }

  // a worker's pipe counters (bg_pipe_stats); 0 if it has none
  int PipeStats(int wid, uint64_t *out, int n) const {
    bg_pipe *p = lanes_[wid].pipe.load(std::memory_order_acquire);
    return p ? bg_pipe_stats(p, out, n) : -1;
  }

  // packets this module holds (submitted, not yet handed on)
  size_t Pending() const {
    size_t n = 0;
    for (const Lane &l : lanes_)
      if (bg_pipe *p = l.pipe.load(std::memory_order_acquire)) n += bg_pipe_pending(p);
    return n;
  }

 protected:
  GpuModule() { max_allowed_workers_ = Worker::kMaxWorkers; }

  CommandResponse Create(const char *mclass, const google::protobuf::Message &arg) {
    const std::string b = arg.SerializeAsString();
    const int rc = bg_module_create(mclass, b.data(), b.size(), &m_);
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    return RegisterAttrs();
  }

  // The metadata attributes the module reads (the attr_name fields of
  // ExactMatch / WildcardMatch: AddFieldOne's AddMetadataAttr,
  // exact_match.cc:78-86, wildcard_match.cc:89-95) registered with bessd,
  // whose pipeline assigns their offsets (Module::attr_offset)
  CommandResponse RegisterAttrs() {
    char name[128];
    uint32_t size = 0;
    int i = 0;
    for (; bg_module_attr(m_, i, name, sizeof(name), &size) > 0; i++) {
      const int r = AddMetadataAttr(name, size, bess::metadata::Attribute::AccessMode::kRead);
      if (r < 0) return CommandFailure(-r, "idx %d: add_metadata_attr() failed", i);
    }
    has_attrs_ = i > 0;
    return CommandSuccess();
  }

  // Create, with the deferred datapath: ProcessBatch enqueues, a task emits
  CommandResponse CreateDeferred(const char *mclass, const google::protobuf::Message &arg,
                                 size_t pipe_batch = kPipeBatch,
                                 int pipe_depth = kPipeDepth) {
    CommandResponse r = Create(mclass, arg);
    if (r.code() != 0) return r;
    pipe_batch_ = pipe_batch;
    pipe_depth_ = pipe_depth;
    if (RegisterTask(nullptr) == INVALID_TASK_ID)
      return CommandFailure(ENOMEM, "Task creation failed");
    deferred_ = true;
    return CommandSuccess();
  }

  // `cmd` with its argument; the C side checks it and answers with the
  // reference's errno and message. resp: the command's response message.
  // (A THREAD_UNSAFE command launches the pipes' partly filled slots
  // first, so queued packets keep the rules they were submitted under.)
  CommandResponse Run(const char *cmd, const google::protobuf::Message &arg,
                      google::protobuf::Message *resp = nullptr) {
    const std::string in = arg.SerializeAsString();
    std::string out(1 << 16, '\0');
    size_t len = out.size();
    int rc = bg_module_command(m_, cmd, in.data(), in.size(), &out[0], &len);
    if (rc == -ENOBUFS && len > out.size()) {  // a larger response (get_*): again
      out.resize(len);
      rc = bg_module_command(m_, cmd, in.data(), in.size(), &out[0], &len);
    }
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    if (!resp) return CommandSuccess();
    resp->ParseFromArray(out.data(), (int)len);
    return CommandSuccess(*resp);
  }

  // bessd's per-call Context as the C ABI's bg_ctx: ctx->current_igate
  // (ACL, StaticNAT, NAT act on it) and ctx->current_ns (NAT's clock) go
  // with the call, never into the shared module
  static bg_ctx CallCtx(const Context *ctx) {
    bg_ctx c;
    c.now_ns = ctx->current_ns;
    c.igate = ctx->current_igate;
    c.device = -1;
    c.wid = (uint32_t)ctx->wid;
    return c;
  }

  // ProcessBatch: the datapath the module was created with
  void Forward(Context *ctx, bess::PacketBatch *batch) {
    if (deferred_)
      Enqueue(ctx, batch);
    else
      ProcessSync(ctx, batch);
  }

  // ProcessBatch on the GPU, synchronously
  void ProcessSync(Context *ctx, bess::PacketBatch *batch) {
    const int n = batch->cnt();
    uint8_t *heads[bess::PacketBatch::kMaxBurst] = {};
    uint8_t *metas[bess::PacketBatch::kMaxBurst] = {};
    uint16_t og[bess::PacketBatch::kMaxBurst];
    for (int i = 0; i < n; i++) {
      heads[i] = batch->pkts()[i]->head_data<uint8_t *>();
      metas[i] = batch->pkts()[i]->metadata<uint8_t *>();
    }
    const bg_ctx c = CallCtx(ctx);
    std::shared_lock<std::shared_mutex> meta(meta_mu_, std::defer_lock);
    if (has_attrs_) {
      if (!AttrsBound() && !Rebind(ctx)) {
        for (int i = 0; i < n; i++) DropPacket(ctx, batch->pkts()[i]);
        return;
      }
      meta.lock();
    }
    if ((has_attrs_ ? bg_module_process_meta(m_, &c, heads, metas, (size_t)n, og)
                    : bg_module_process(m_, &c, heads, (size_t)n, og)) < 0) {
      for (int i = 0; i < n; i++) DropPacket(ctx, batch->pkts()[i]);
      return;
    }
    for (int i = 0; i < n; i++) Emit(ctx, batch->pkts()[i], og[i]);
  }

  // ProcessBatch, deferred: the batch joins this worker's pipe, then what
  // has finished there leaves
  void Enqueue(Context *ctx, bess::PacketBatch *batch) {
    std::shared_lock<std::shared_mutex> meta(meta_mu_, std::defer_lock);
    if (has_attrs_) {  // the metadata layout the pipes stage with is current
      if (!AttrsBound() && !Rebind(ctx)) {
        for (int i = 0; i < batch->cnt(); i++) DropPacket(ctx, batch->pkts()[i]);
        return;
      }
      meta.lock();
    }
    Lane &l = lanes_[ctx->wid];
    l.in_call.store(true);  // (seq_cst: pairs with RunTask's claim)
    while (l.draining.load(std::memory_order_acquire)) {
    }
    EnqueueOwned(ctx, batch, l);
    l.in_call.store(false, std::memory_order_release);
  }

  // Whether the attribute offsets bessd assigned are the ones bound into the
  // library (bessd recomputes them when the pipeline changes, workers paused)
  bool AttrsBound() const {
    const size_t n = all_attrs().size();
    if (nbound_.load(std::memory_order_acquire) != (int)n) return false;
    for (size_t i = 0; i < n; i++)
      if (bound_[i].load(std::memory_order_relaxed) != (int32_t)attr_offset(i)) return false;
    return true;
  }

  // Bind the current offsets (first batch, or after a pipeline change): every
  // worker's pipe -- staged with the old layout -- is drained (its packets
  // leave here, in order) and closed; workers open new ones. false: the
  // library refused the layout (an attribute no upstream module writes,
  // where the reference would dereference a null attribute pointer).
  bool Rebind(Context *ctx) {
    std::unique_lock<std::shared_mutex> lk(meta_mu_);
    if (AttrsBound()) return true;
    for (Lane &l : lanes_) {
      bg_pipe *p = l.pipe.exchange(nullptr);
      if (!p) continue;
      (void)bg_pipe_flush(p);
      void *ck[256];
      uint16_t g[256];
      long k;
      while ((k = bg_pipe_poll(p, 1, ck, g, 256)) > 0)
        for (long i = 0; i < k; i++) Emit(ctx, static_cast<bess::Packet *>(ck[i]), g[i]);
      bg_pipe_destroy(p);
    }
    const size_t n = all_attrs().size();
    std::vector<const char *> names(n);
    std::vector<int32_t> offs(n);
    for (size_t i = 0; i < n; i++) {
      names[i] = all_attrs()[i].name.c_str();
      offs[i] = attr_offset(i);
    }
    nbound_.store(-1, std::memory_order_relaxed);
    if (bg_module_bind_meta(m_, -1, names.data(), offs.data(), (int)n) < 0) return false;
    for (size_t i = 0; i < n; i++) bound_[i].store(offs[i], std::memory_order_relaxed);
    nbound_.store((int)n, std::memory_order_release);
    return true;
  }

  void EnqueueOwned(Context *ctx, bess::PacketBatch *batch, Lane &l) {
    const int n = batch->cnt();
    bg_pipe *p = l.pipe.load(std::memory_order_acquire);
    if (!p && !(p = OpenLane(ctx->wid))) {
      for (int i = 0; i < n; i++) DropPacket(ctx, batch->pkts()[i]);
      return;
    }
    uint8_t *heads[bess::PacketBatch::kMaxBurst] = {};
    uint8_t *metas[bess::PacketBatch::kMaxBurst] = {};
    uint16_t lens[bess::PacketBatch::kMaxBurst] = {};
    // the packets' mbuf lines in flight together (head_data() reads them),
    // then, as each arrives, the line of its data the pipe gathers from
    for (int i = 0; i < n; i++) __builtin_prefetch(batch->pkts()[i]);
    for (int i = 0; i < n; i++) {
      bess::Packet *pkt = batch->pkts()[i];
      heads[i] = pkt->head_data<uint8_t *>();
      lens[i] = pkt->data_len();
      __builtin_prefetch(heads[i] + l.win_lo);
      if (has_attrs_) metas[i] = pkt->metadata<uint8_t *>();
    }
    const bg_ctx c = CallCtx(ctx);
    void *const *ck = reinterpret_cast<void *const *>(batch->pkts());
    if ((has_attrs_ ? bg_pipe_submit_meta(p, &c, heads, metas, lens, ck, (size_t)n)
                    : bg_pipe_submit(p, &c, heads, lens, ck, (size_t)n)) < 0) {
      for (int i = 0; i < n; i++) DropPacket(ctx, batch->pkts()[i]);
      return;
    }
    l.submits.fetch_add(1, std::memory_order_relaxed);
    Drain(ctx, p);
  }

  // a gate per packet: BG_GATE_NONE leaves the packet alone (the module did
  // not emit it), BG_DROP_GATE drops it, any other gate goes to EmitPacket
  void Emit(Context *ctx, bess::Packet *pkt, uint16_t g) {
    if (g == BG_GATE_NONE) return;
    if (g >= BG_MAX_GATES)
      DropPacket(ctx, pkt);
    else
      EmitPacket(ctx, pkt, g);
  }

  std::string Desc() const {
    char b[256] = "";
    if (m_) bg_module_desc(m_, b, sizeof(b));
    return b;
  }

  bg_module *m_ = nullptr;

 private:
  // the worker's pipe, on device wid % (visible devices): the workers of one
  // process spread over its GPUs, each using the module's table replica there
  // process-wide reference counts of the registered pool chunks: +1 / -1
  static void PoolRegion(void *base, size_t len, int delta) {
    static std::mutex mu;
    static std::vector<std::pair<void *, int>> refs;
    std::lock_guard<std::mutex> lk(mu);
    for (size_t i = 0; i < refs.size(); i++) {
      if (refs[i].first != base) continue;
      if ((refs[i].second += delta) == 0) {
        (void)bg_host_unregister(base);
        refs.erase(refs.begin() + (long)i);
      }
      return;
    }
    if (delta > 0 && bg_host_register(base, len) == 0) refs.emplace_back(base, 1);
  }

  void RegisterPool() {
    bess::PacketPool *pool = bess::PacketPool::GetDefaultPool(current_worker.socket());
    if (!pool) return;
    rte_mempool_mem_iter(
        pool->pool(),
        [](rte_mempool *, void *self, rte_mempool_memhdr *h, unsigned) {
          GpuModule *m = static_cast<GpuModule *>(self);
          for (void *b : m->registered_)
            if (b == h->addr) return;
          PoolRegion(h->addr, h->len, 1);
          m->registered_.push_back(h->addr);
        },
        this);
  }

  bg_pipe *OpenLane(int wid) {
    if (in_place_) {  // (workers open their lanes one at a time: lanes_mu_)
      std::lock_guard<std::mutex> lk(lanes_mu_);
      RegisterPool();
    }
    const int nd = bg_device_count();
    bg_pipe *p = nullptr;
    // within the budget, full-size slots first (each slot costs a submit or
    // a launch), then as many in flight as fit, at least two
    const size_t budget = PipeBudget();
    int depth = pipe_depth_;
    if (budget / (size_t)depth < pipe_batch_)
      depth = (int)std::max<size_t>(2, std::min<size_t>((size_t)depth, budget / pipe_batch_));
    const size_t batch = std::min(pipe_batch_, std::max<size_t>(32, budget / (size_t)depth));
    if (nd <= 0 || bg_pipe_create(m_, wid % nd, batch, depth, 0, &p) < 0)
      return nullptr;
    int lo = 0, hi = 0;
    size_t stride = 0;
    if (bg_pipe_window(p, &lo, &hi, &stride) == 0 && lo > 0) lanes_[wid].win_lo = lo;
    lanes_[wid].pipe.store(p, std::memory_order_release);
    return p;
  }

  // emit the pipe's finished packets (in submission order); each packet's
  // mbuf line is fetched a few packets ahead for the module downstream
  uint32_t Drain(Context *ctx, bg_pipe *p) {
    void *ck[512];
    uint16_t g[512];
    uint32_t total = 0;
    long k;
    while ((k = bg_pipe_poll(p, 0, ck, g, 512)) > 0) {
      for (long i = 0; i < k && i < 8; i++) __builtin_prefetch(ck[i]);
      for (long i = 0; i < k; i++) {
        if (i + 8 < k) __builtin_prefetch(ck[i + 8]);
        Emit(ctx, static_cast<bess::Packet *>(ck[i]), g[i]);
      }
      total += (uint32_t)k;
      if (k < 512) break;
    }
    return total;
  }

  bool deferred_ = false;
  // attr_name fields: the offsets bound into the library (AttrsBound); the
  // datapath holds meta_mu_ shared, a re-bind exclusively
  bool has_attrs_ = false;
  std::shared_mutex meta_mu_;
  std::atomic<int> nbound_{-1};
  std::atomic<int32_t> bound_[16] = {};
  size_t pipe_batch_ = kPipeBatch;
  int pipe_depth_ = kPipeDepth;
  bool in_place_ = false;             // UsePacketPoolInPlace
  std::mutex lanes_mu_;               // RegisterPool from the workers' first calls
  std::vector<void *> registered_;    // the pool chunks this module registered
  Lane lanes_[Worker::kMaxWorkers];
};

#endif  // BESS_MODULES_GPU_MODULE_H_
