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
//     swap                        turn each IPv4 TCP/UDP frame into its reply
//                                 (addresses and ports exchanged; checksums
//                                 unchanged, the sums being symmetric)
//     process <igate> <now_ns>    ProcessBatch over the frames, 32 at a time
//                                 -> "out" + per packet: gate, D (dropped)
//                                    or - (not emitted); "data <hex>" per
//                                    packet's first 64 bytes afterwards
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "core/module.h"

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

static int run() {
  Module *m = nullptr;
  const ModuleClass *cls = nullptr;
  std::vector<uint8_t *> bufs;
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
    } else if (op == "connect") {
      int g;
      in >> g;
      m->ConnectOGate((gate_idx_t)g);
    } else if (op == "frames") {
      std::string path;
      size_t stride, n;
      in >> path >> stride >> n;
      std::ifstream f(path, std::ios::binary);
      std::vector<char> fr(stride);
      for (size_t i = 0; i < n; i++) {
        f.read(fr.data(), (std::streamsize)stride);
        uint8_t *b = static_cast<uint8_t *>(aligned_alloc(64, SNBUF_SIZE));
        memset(b, 0, SNBUF_SIZE);
        bess::Packet *p = new (b) bess::Packet();
        memcpy(p->head_data<uint8_t *>(), fr.data(), stride);
        p->set_total_len((uint32_t)stride);
        p->set_data_len((uint16_t)stride);
        bufs.push_back(b);
      }
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
      std::map<bess::Packet *, std::string> out;
      for (size_t b0 = 0; b0 < bufs.size(); b0 += bess::PacketBatch::kMaxBurst) {
        bess::PacketBatch batch;
        for (size_t i = b0; i < bufs.size() && i < b0 + bess::PacketBatch::kMaxBurst; i++)
          batch.add(reinterpret_cast<bess::Packet *>(bufs[i]));
        Context ctx;
        ctx.current_igate = (gate_idx_t)ig;
        ctx.current_ns = now;
        m->ProcessBatch(&ctx, &batch);
        for (auto &e : ctx.emitted) out[e.first] = std::to_string(e.second);
        for (auto *p : ctx.dropped) out[p] = "D";
      }
      printf("out");
      for (uint8_t *b : bufs) {
        auto it = out.find(reinterpret_cast<bess::Packet *>(b));
        printf(" %s", it == out.end() ? "-" : it->second.c_str());
      }
      printf("\n");
      for (uint8_t *b : bufs) {
        bess::Packet *p = reinterpret_cast<bess::Packet *>(b);
        printf("data %u %s\n", p->total_len(),
               hex(std::string(p->head_data<const char *>(), 64)).c_str());
      }
    }
    fflush(stdout);
  }
  if (m) {
    m->DeInit();
    delete m;
  }
  for (uint8_t *b : bufs) free(b);
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && !strcmp(argv[1], "dump")) return dump();
  if (argc > 1 && !strcmp(argv[1], "run")) return run();
  fprintf(stderr, "usage: drive dump | run < script\n");
  return 2;
}
