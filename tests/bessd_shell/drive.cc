// Test driver for the bessd plugin wrappers (integration/bessd/*_gpu.cc)
// compiled against the header shell in tests/bessd_shell/core.
//
//   drive dump            every registered class as JSON: name template,
//                         help, gate counts, commands table
//   drive run < script    one module driven through its wrapper:
//     create <Class> <hex Arg>    Init            -> "rc <code> <msg>"
//     cmd <name> <hex Arg>        a command       -> "rc <code> <msg> <hex resp>"
//     desc                        GetDesc         -> "desc <text>"
//     connect <ogate>             ConnectModules for that output gate
//     frames <path> <stride> <n>  n frames of `stride` bytes into snbufs
//     lens <path>                 each packet's data_len (and total_len): one
//                                 u16 per packet (the bytes past it keep the
//                                 frames file's, as a reused buffer would)
//     meta <path> <bytes>         each packet's metadata area (Packet::metadata,
//                                 SNBUF_METADATA_OFF) gets `bytes` bytes from
//                                 the file, packet after packet
//     attr_offset <id> <off>      place the module's attribute `id` at metadata
//                                 offset `off` (Pipeline::ComputeMetadataOffsets)
//     swap                        turn each IPv4 TCP/UDP frame into its reply
//                                 (addresses and ports exchanged; checksums
//                                 unchanged, the sums being symmetric)
//     process <igate> <now_ns>    ProcessBatch over the frames, 32 at a time,
//                                 then the module's task until it holds no
//                                 packet -> "out" + per packet: gate, D
//                                 (dropped) or - (not emitted); "data <hex>"
//                                 per packet's first 64 bytes afterwards
//     pool <capacity>             a packet pool of `capacity` snbufs (bessd's
//                                 --buffers, core/opts.cc:127): `pipeline`
//                                 then allocates every Source batch from it
//                                 (AllocBulk; a Source finding it empty
//                                 waits) and copies the frame in, as Source
//                                 does with its template, and the Sink frees
//                                 each packet back (Packet::Free)
//     pipeline <workers> <reps> <igate> <now_ns> <verify>
//                                 Source -> module -> Sink on `workers`
//                                 threads (pinned), each over its own slice
//                                 of the frames `reps` times in 32-packet
//                                 batches (wid = worker); worker 0 also runs
//                                 the module's task (every 64 batches, then
//                                 until the module holds no packet); with a
//                                 pool: "pool <available> <capacity>
//                                 <source_waits>" afterwards
//                                 -> "pipeline <Mpps> <seconds> <packets>",
//                                 "out" as above for the last pass, and with
//                                 verify "order ok|bad": each worker's
//                                 emitted packets left in the order they
//                                 came in (hence per gate, module.h:268-272)
//     cpu_em <keys> <gates> <n> <stride>  the CPU baseline's table: the
//                                 oracle's restatement of ExactMatch (5-tuple
//                                 fields), n rules (keys `stride` bytes
//                                 apart in gather_key layout, u16 gates)
//     sleep <ms>                  pause (after a warm pass: the module's
//                                 run-time compile finishes untimed)
//     cpu_wm <keys> <masks> <prios> <gates> <n>  the same for WildcardMatch
//                                 (16-byte keys and masks, i32 priorities)
//     cpu_l4 <verify>             the same for L4Checksum (in place)
//     pipeline_cpu <workers> <reps>  the same Source -> Sink loop with the
//                                 restated reference ProcessBatch on the CPU
//                                 in the middle (head_data() per packet,
//                                 MakeKeys + CuckooMap Find, EmitPacket with
//                                 the created module's connected gates) --
//                                 the cpu_baseline in the same harness
#include <execinfo.h>

#include <chrono>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>
#include <x86intrin.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "core/module.h"
#include "core/modules/gpu_module.h"
#include "oracle.h"  // test infrastructure: the CPU baseline (pipeline_cpu)

// mempool object stride: the snbuf plus the mempool's object header, so
// head_data() sits at +512 of a 2624-byte object (core/snbuf_layout.h)
static const size_t kObj = SNBUF_SIZE + 64;

static double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static std::string json_str(const std::string &s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o + "\"";
}

static std::string unhex(const std::string &h) {
  std::string o;
  if (h == "-") return o;
  for (size_t i = 0; i + 1 < h.size(); i += 2) o += (char)strtol(h.substr(i, 2).c_str(), 0, 16);
  return o;
}

static std::string hex(const std::string &b) {
  static const char *d = "0123456789abcdef";
  std::string o;
  for (unsigned char c : b) {
    o += d[c >> 4];
    o += d[c & 15];
  }
  return o.empty() ? "-" : o;
}

static int dump() {
  printf("{");
  bool first = true;
  for (auto &kv : module_classes()) {
    const ModuleClass &c = kv.second;
    printf("%s%s: {\"name_template\": %s, \"help\": %s, \"igates\": %d, \"ogates\": %d, "
           "\"cmds\": [",
           first ? "" : ", ", json_str(kv.first).c_str(), json_str(c.name_template).c_str(),
           json_str(c.help).c_str(), c.igates, c.ogates);
    first = false;
    for (size_t i = 0; i < c.cmds.size(); i++)
      printf("%s[%s, %s, %s]", i ? ", " : "", json_str(c.cmds[i].cmd).c_str(),
             json_str(c.cmds[i].arg_type).c_str(),
             c.cmds[i].mt_safe == Command::THREAD_SAFE ? "\"THREAD_SAFE\"" : "\"THREAD_UNSAFE\"");
    printf("]}");
  }
  printf("}\n");
  return 0;
}

static void print_rc(const CommandResponse &r, bool data) {
  printf("rc %d %s", r.code(), r.errmsg().empty() ? "-" : r.errmsg().c_str());
  if (data) printf(" %s", hex(r.data()).c_str());
  printf("\n");
}

// The module's task until it holds no packet (deferred plugins), or once.
static void run_task(Module *m, Context *ctx) {
  GpuModule *g = dynamic_cast<GpuModule *>(m);
  if (!m->is_task()) return;
  do {
    m->RunTask(ctx, nullptr, nullptr);
  } while (g && g->Pending() > 0);
}

struct Sink {  // where a worker's emitted and dropped packets go
  std::vector<std::string> *gate = nullptr;  // per packet (verify)
  std::vector<uint16_t> *fast = nullptr;     // per packet (timing)

  uint8_t *pool = nullptr;
  bool free_packets = false;  // pool mode: each packet goes back (Packet::Free)
  uint64_t n = 0;
  void take(Context &ctx) {
    for (auto &e : ctx.emitted) put(e.first, e.second);
    for (auto *p : ctx.dropped) put(p, 0xFFFF);
    n += ctx.emitted.size() + ctx.dropped.size();
    if (free_packets) {
      for (auto &e : ctx.emitted) bess::Packet::Free(e.first);
      for (auto *p : ctx.dropped) bess::Packet::Free(p);
    }
    ctx.emitted.clear();
    ctx.dropped.clear();
  }
  void put(bess::Packet *p, uint32_t g) {
    const size_t i = p->pool_index();
    if (fast) (*fast)[i] = (uint16_t)g;
    if (gate) (*gate)[i] = g == 0xFFFF ? "D" : std::to_string(g);
  }
};

static void pin(int w) {
  cpu_set_t set;
  std::vector<int> cpus;
  if (sched_getaffinity(0, sizeof(set), &set) == 0)
    for (int c = 0; c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &set)) cpus.push_back(c);
  if (cpus.empty()) return;
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(cpus[(size_t)w % cpus.size()], &one);
  pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
}

static int run() {
  Module *m = nullptr;
  const ModuleClass *cls = nullptr;
  uint8_t *pool = nullptr;
  or_em *cpu_em = nullptr;
  or_wm *cpu_wm = nullptr;
  int cpu_l4 = -1;  // L4Checksum's verify flag (cpu_l4), -1: none
  std::vector<uint8_t *> bufs;
  std::vector<char> fdata;  // the frames file (pool mode: the Sources' frames)
  size_t fstride = 0;
  // each frame's length (Ethernet + the IPv4 total length, within the
  // slot): what pool mode's Source copies per packet, as the reference's
  // Source copies its pkt_size-byte template
  std::vector<uint16_t> flen;
  bess::PacketPool *ppool = nullptr;
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream in(line);
    std::string op;
    in >> op;
    if (op == "create") {
      std::string name, h;
      in >> name >> h;
      auto it = module_classes().find(name);
      if (it == module_classes().end()) {
        printf("rc 2 no such class\n");
        continue;
      }
      cls = &it->second;
      m = cls->make();
      google::protobuf::Any a;
      a.ParseFromString(unhex(h));
      print_rc(cls->init(m, a), false);
    } else if (op == "cmd") {
      std::string name, h;
      in >> name >> h;
      bool found = false;
      for (const Command &c : cls->cmds) {
        if (c.cmd != name) continue;
        google::protobuf::Any a;
        a.ParseFromString(unhex(h));
        print_rc(c.func(m, a), true);
        found = true;
      }
      if (!found) printf("rc 95 no such command\n");
    } else if (op == "desc") {
      printf("desc %s\n", m->GetDesc().c_str());
    } else if (op == "sleep") {  // ms: lets a module's background work
                                  // (a run-time compile) finish untimed
      int ms;
      in >> ms;
      std::this_thread::sleep_for(std::chrono::milliseconds(ms));
    } else if (op == "connect") {
      int g;
      in >> g;
      m->ConnectOGate((gate_idx_t)g);
    } else if (op == "frames") {
      std::string path;
      size_t stride, n;
      in >> path >> stride >> n;
      std::ifstream f(path, std::ios::binary);
      fdata.assign(n * stride, 0);
      f.read(fdata.data(), (std::streamsize)(n * stride));
      fstride = stride;
      flen.assign(n, (uint16_t)std::min<size_t>(stride, 0xFFFF));
      for (size_t i = 0; i < n; i++) {
        const uint8_t *fr = reinterpret_cast<const uint8_t *>(fdata.data() + i * stride);
        if (stride >= 18 && fr[12] == 0x08 && fr[13] == 0x00) {
          const size_t l = 14 + ((size_t)fr[16] << 8 | fr[17]);
          flen[i] = (uint16_t)std::max<size_t>(60, std::min(l, stride));
        }
      }
      free(pool);
      bufs.clear();
      pool = static_cast<uint8_t *>(aligned_alloc(64, n * kObj));
      memset(pool, 0, n * kObj);
      for (size_t i = 0; i < n; i++) {
        const char *fr = fdata.data() + i * stride;
        uint8_t *b = pool + i * kObj;
        bess::Packet *p = new (b) bess::Packet();
        p->set_pool_index((uint32_t)i);
        memcpy(p->head_data<uint8_t *>(), fr, stride);
        p->set_total_len((uint32_t)stride);
        p->set_data_len((uint16_t)stride);
        bufs.push_back(b);
      }
    } else if (op == "lens") {
      std::string path;
      in >> path;
      std::ifstream f(path, std::ios::binary);
      for (uint8_t *b : bufs) {
        uint16_t l = 0;
        f.read(reinterpret_cast<char *>(&l), 2);
        bess::Packet *p = reinterpret_cast<bess::Packet *>(b);
        p->set_total_len(l);
        p->set_data_len(l);
      }
    } else if (op == "cpu_l4") {
      in >> cpu_l4;
      printf("cpu_l4 %d\n", cpu_l4);
    } else if (op == "pool") {
      size_t cap;
      in >> cap;
      delete ppool;
      ppool = new bess::PacketPool(cap);
      bess::PacketPool::default_pool() = ppool;
    } else if (op == "meta") {
      std::string path;
      size_t nb;
      in >> path >> nb;
      std::ifstream f(path, std::ios::binary);
      std::vector<char> md(nb);
      for (uint8_t *b : bufs) {
        f.read(md.data(), (std::streamsize)nb);
        memcpy(reinterpret_cast<bess::Packet *>(b)->metadata<uint8_t *>(), md.data(),
               std::min<size_t>(nb, SNBUF_METADATA));
      }
    } else if (op == "attr_offset") {
      int id, off;
      in >> id >> off;
      m->set_attr_offset((size_t)id, (bess::metadata::mt_offset_t)off);
    } else if (op == "swap") {
      for (uint8_t *b : bufs) {
        uint8_t *f = reinterpret_cast<bess::Packet *>(b)->head_data<uint8_t *>();
        const int l4 = 14 + 4 * (f[14] & 15);
        for (int i = 0; i < 4; i++) std::swap(f[26 + i], f[30 + i]);
        for (int i = 0; i < 2; i++) std::swap(f[l4 + i], f[l4 + 2 + i]);
      }
    } else if (op == "process") {
      int ig;
      unsigned long long now;
      in >> ig >> now;
      std::vector<std::string> out(bufs.size(), "-");
      Sink sink;
      sink.gate = &out;
      sink.pool = pool;
      Context ctx;
      ctx.current_igate = (gate_idx_t)ig;
      ctx.current_ns = now;
      for (size_t b0 = 0; b0 < bufs.size(); b0 += bess::PacketBatch::kMaxBurst) {
        bess::PacketBatch batch;
        for (size_t i = b0; i < bufs.size() && i < b0 + bess::PacketBatch::kMaxBurst; i++)
          batch.add(reinterpret_cast<bess::Packet *>(bufs[i]));
        m->ProcessBatch(&ctx, &batch);
        sink.take(ctx);
      }
      run_task(m, &ctx);
      sink.take(ctx);
      printf("out");
      for (auto &g : out) printf(" %s", g.c_str());
      printf("\n");
      for (uint8_t *b : bufs) {
        bess::Packet *p = reinterpret_cast<bess::Packet *>(b);
        printf("data %u %s\n", p->total_len(),
               hex(std::string(p->head_data<const char *>(), 64)).c_str());
      }
    } else if (op == "cpu_em") {
      std::string kp, gp;
      size_t nr, ks = 16;
      in >> kp >> gp >> nr >> ks;
      std::vector<uint8_t> keys(nr * ks);
      std::vector<uint16_t> gates(nr);
      std::ifstream fk(kp, std::ios::binary), fg(gp, std::ios::binary);
      fk.read(reinterpret_cast<char *>(keys.data()), (std::streamsize)keys.size());
      fg.read(reinterpret_cast<char *>(gates.data()), (std::streamsize)(nr * 2));
      if (cpu_em) or_em_free(cpu_em);
  if (cpu_wm) or_wm_free(cpu_wm);
      cpu_em = or_em_new();
      const int fo[5] = {23, 26, 30, 34, 36}, fs[5] = {1, 4, 4, 2, 2};
      for (int i = 0; i < 5; i++) or_em_add_field(cpu_em, fo[i], fs[i], 0, i, nullptr, 0);
      printf("cpu_em %d\n", or_em_add_rules(cpu_em, keys.data(), nr, ks, gates.data()));
    } else if (op == "cpu_wm") {
      // keys / masks: n x 16 bytes (the 13-byte 5-tuple key, zero padded),
      // priorities n x int32, gates n x u16
      std::string kp, mp, pp, gp;
      size_t nr;
      in >> kp >> mp >> pp >> gp >> nr;
      std::vector<uint8_t> keys(nr * 16), masks(nr * 16);
      std::vector<int32_t> prio(nr);
      std::vector<uint16_t> gates(nr);
      std::ifstream fk(kp, std::ios::binary), fm(mp, std::ios::binary),
          fp(pp, std::ios::binary), fg(gp, std::ios::binary);
      fk.read(reinterpret_cast<char *>(keys.data()), (std::streamsize)keys.size());
      fm.read(reinterpret_cast<char *>(masks.data()), (std::streamsize)masks.size());
      fp.read(reinterpret_cast<char *>(prio.data()), (std::streamsize)(nr * 4));
      fg.read(reinterpret_cast<char *>(gates.data()), (std::streamsize)(nr * 2));
      if (cpu_wm) or_wm_free(cpu_wm);
      cpu_wm = or_wm_new();
      const int fo[5] = {23, 26, 30, 34, 36}, fs[5] = {1, 4, 4, 2, 2};
      for (int i = 0; i < 5; i++) or_wm_add_field(cpu_wm, fo[i], fs[i], nullptr, 0);
      or_wm_init_done(cpu_wm);
      int rc = 0;
      for (size_t i = 0; i < nr && !rc; i++) {
        uint8_t k[OR_KEY_BYTES] = {}, m[OR_KEY_BYTES] = {};
        memcpy(k, &keys[i * 16], 16);
        memcpy(m, &masks[i * 16], 16);
        rc = or_wm_add(cpu_wm, k, m, prio[i], gates[i]);
      }
      printf("cpu_wm %d\n", rc);
    } else if (op == "pipeline" || op == "pipeline_cpu") {
      const bool cpu = op == "pipeline_cpu";
      int nw, reps, ig = 0, verify = 0;
      unsigned long long now = 0;
      in >> nw >> reps;
      if (!cpu) in >> ig >> now >> verify;
      if (cpu && !cpu_em && !cpu_wm && cpu_l4 < 0) {
        printf("rc 22 cpu_em / cpu_wm / cpu_l4 first\n");
        continue;
      }
      const size_t n = bufs.size();
      num_workers = nw;
      std::atomic<uint64_t> source_waits{0};
      std::vector<std::string> out(n, "-");
      std::vector<uint16_t> fast(n, 0xFFFE);
      std::vector<uint64_t> seq(n, ~0ull);
      std::atomic<uint64_t> counter{0};
      std::atomic<int> started{0}, finished{0};
      std::atomic<bool> go{false};
      std::vector<uint64_t> sunk(nw, 0);
      uint64_t tsc[4] = {0, 0, 0, 0};
      double t0 = 0, t1 = 0;
      const uint64_t tsc0 = __rdtsc();
      auto worker = [&](int w) {
        pin(w);
        Sink sink;
        sink.pool = pool;
        sink.free_packets = ppool != nullptr;
        Context ctx;
        if (verify) {
          sink.gate = &out;
          // (only emitted packets carry an emission number: drops go to
          // the dead batch)
          ctx.emit_seq = &seq;
          ctx.emit_counter = &counter;
        } else {
          sink.fast = &fast;
        }
        ctx.wid = w;
        ctx.current_igate = (gate_idx_t)ig;
        ctx.current_ns = now;
        ctx.emitted.reserve(1 << 16);
        const size_t lo = n * w / nw, hi = n * (w + 1) / nw;
        started++;
        while (!go.load()) {
        }
        uint64_t nb = 0;
        uint64_t c_src = 0, c_proc = 0, c_sink = 0, c_task = 0;  // TSC cycles per phase
        for (int r = 0; r < reps; r++)
          for (size_t b0 = lo; b0 < hi; b0 += bess::PacketBatch::kMaxBurst) {
            bess::PacketBatch batch;  // the Source's batch
            const size_t cnt = std::min(hi - b0, (size_t)bess::PacketBatch::kMaxBurst);
            const uint64_t cs = __rdtsc();
            if (ppool) {
              // packets from the pool, each filled with its frame (Source
              // copies its template the same way); an empty pool: wait
              // for the Sinks (worker 0 keeps running the module's task)
              bess::Packet *pk[bess::PacketBatch::kMaxBurst];
              while (!ppool->AllocBulk(pk, cnt, fstride)) {
                source_waits++;
                if (!cpu && w == 0 && m->is_task()) {
                  m->RunTask(&ctx, nullptr, nullptr);
                  sink.take(ctx);
                }
                std::this_thread::yield();
              }
              for (size_t j = 0; j < cnt; j++) {
                const uint16_t fl = flen[b0 + j];
                memcpy(pk[j]->head_data<uint8_t *>(), fdata.data() + (b0 + j) * fstride, fl);
                pk[j]->set_total_len(fl);
                pk[j]->set_data_len(fl);
                pk[j]->set_pool_index((uint32_t)(b0 + j));
                batch.add(pk[j]);
              }
            } else {
              for (size_t i = b0; i < b0 + cnt; i++)
                batch.add(reinterpret_cast<bess::Packet *>(pool + i * kObj));
            }
            const uint64_t c0 = __rdtsc();
            c_src += c0 - cs;
            if (cpu) {  // ExactMatch::ProcessBatch restated (exact_match.cc:224-244)
                        // or WildcardMatch's (cpu_wm), L4Checksum's (cpu_l4)
              uint8_t *heads[bess::PacketBatch::kMaxBurst];
              uint16_t g[bess::PacketBatch::kMaxBurst];
              for (int i = 0; i < batch.cnt(); i++)
                heads[i] = batch.pkts()[i]->head_data<uint8_t *>();
              if (cpu_l4 >= 0)  // L4Checksum::ProcessBatch (l4_checksum.cc:41-83)
                or_l4_checksum_batch(heads, batch.cnt(), cpu_l4, g);
              else if (cpu_wm)  // WildcardMatch::ProcessBatch (wildcard_match.cc:159-203)
                or_wm_process_batch(cpu_wm, heads, batch.cnt(), DROP_GATE, g);
              else
                or_em_process_batch(cpu_em, heads, batch.cnt(), DROP_GATE, g);
              for (int i = 0; i < batch.cnt(); i++)
                if (g[i] != OR_GATE_NONE) m->EmitPacket(&ctx, batch.pkts()[i], g[i]);
            } else {
              m->ProcessBatch(&ctx, &batch);
            }
            const uint64_t c1 = __rdtsc();
            sink.take(ctx);
            const uint64_t c2 = __rdtsc();
            c_proc += c1 - c0;
            c_sink += c2 - c1;
            if (!cpu && w == 0 && (++nb & 63) == 0 && m->is_task()) {
              m->RunTask(&ctx, nullptr, nullptr);
              sink.take(ctx);
              c_task += __rdtsc() - c2;
            }
          }
        finished++;
        if (w == 0) {  // the task's worker: until every worker is done
          while (finished.load() < nw) {
            if (!cpu && m->is_task()) m->RunTask(&ctx, nullptr, nullptr);
            sink.take(ctx);
          }
          if (!cpu) run_task(m, &ctx);
          sink.take(ctx);
          t1 = now_s();
        }
        sunk[w] = sink.n;
        if (ppool) ppool->FlushThreadCache();
        if (w == 0) {
          tsc[0] = c_proc;
          tsc[1] = c_sink;
          tsc[2] = c_task;
          tsc[3] = c_src;
        }
      };
      std::vector<std::thread> th;
      for (int w = 0; w < nw; w++) th.emplace_back(worker, w);
      while (started.load() < nw) {
      }
      t0 = now_s();
      go = true;
      for (auto &t : th) t.join();
      const double dt = t1 - t0;
      const double pk = (double)n * reps;
      printf("pipeline %.3f %.6f %.0f\n", pk / dt / 1e6, dt, pk);
      // worker 0's cycles per packet of its own: ProcessBatch, Sink, task,
      // and the Source's allocation and frame copy (pool runs)
      const double ghz = (double)(__rdtsc() - tsc0) / (now_s() - t0 + 1e-12) / 1e9;
      const double p0 = pk / nw;
      printf("cycles w0 proc %.1f sink %.1f task %.1f source %.1f per_pkt tsc_ghz %.2f\n",
             tsc[0] / p0, tsc[1] / p0, tsc[2] / p0, tsc[3] / p0, ghz);
      printf("out");
      for (size_t i = 0; i < n; i++) {
        if (verify)
          printf(" %s", out[i].c_str());
        else
          printf(" %s", fast[i] == 0xFFFE ? "-" : fast[i] == 0xFFFF ? "D"
                                                 : std::to_string(fast[i]).c_str());
      }
      printf("\n");
      if (ppool)
        printf("pool %zu %zu %llu\n", ppool->Size(), ppool->Capacity(),
               (unsigned long long)source_waits.load());
      if (GpuModule *g = dynamic_cast<GpuModule *>(m)) {
        uint64_t st[16];
        if (g->PipeStats(0, st, 16) == 0)
          printf("stats submits %llu pkts %llu launches %llu launch_ms %.3f full_ms %.3f "
                 "wait_ms %.3f batch %llu submit_cyc_per_pkt %.1f poll_cyc_per_pkt %.1f "
                 "slot_latency_us avg %.1f max %.1f call_ms h2d %.3f kernel %.3f "
                 "gates %.3f lines %.3f done %.3f\n",
                 (unsigned long long)st[0], (unsigned long long)st[1],
                 (unsigned long long)st[2], st[3] * 1e-6, st[4] * 1e-6, st[5] * 1e-6,
                 (unsigned long long)st[6], st[7] / (double)(st[1] ? st[1] : 1),
                 st[8] / (double)(st[1] ? st[1] : 1),
                 st[9] / (double)(st[2] ? st[2] : 1) / 3300.0, st[10] / 3300.0,
                 st[11] * 1e-6, st[12] * 1e-6, st[13] * 1e-6, st[14] * 1e-6,
                 st[15] * 1e-6);
      }
      if (verify) {
        bool ok = true;
        for (int w = 0; w < nw && ok; w++) {
          uint64_t last = 0;
          bool first = true;
          for (size_t i = n * w / nw; i < n * (w + 1) / nw; i++) {
            if (seq[i] == ~0ull) continue;
            if (!first && seq[i] <= last) ok = false;
            last = seq[i];
            first = false;
          }
        }
        printf("order %s\n", ok ? "ok" : "bad");
      }
    }
    fflush(stdout);
  }
  if (m) {
    m->DeInit();
    delete m;
  }
  free(pool);
  bess::PacketPool::default_pool() = nullptr;
  delete ppool;
  if (cpu_em) or_em_free(cpu_em);
  if (cpu_wm) or_wm_free(cpu_wm);
  return 0;
}

// a fatal signal prints the faulting thread's stack (test diagnostics)
static void on_fatal(int sig) {
  void *frames[64];
  const int n = backtrace(frames, 64);
  fprintf(stderr, "drive: signal %d\n", sig);
  backtrace_symbols_fd(frames, n, 2);
  _exit(128 + sig);
}

int main(int argc, char **argv) {
  signal(SIGSEGV, on_fatal);
  signal(SIGBUS, on_fatal);
  if (argc > 1 && !strcmp(argv[1], "dump")) return dump();
  if (argc > 1 && !strcmp(argv[1], "run")) return run();
  fprintf(stderr, "usage: drive dump | run < script\n");
  return 2;
}
