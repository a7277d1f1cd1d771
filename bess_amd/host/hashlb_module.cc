// hashlb_module.cc -- HashLB (core/modules/hash_lb.{h,cc}) with its
// ProcessBatch on the GPU (bg_hlb_*, bg_lb.hip hlb_kernel).
//
// Same class name, commands table, Init argument, error codes and messages
// and GetDesc as the reference, including its partial-update behaviour:
// set_gates writes gates_[i] as it validates (an invalid gate leaves the
// earlier entries written and num_gates_ unchanged), and a failing
// set_mode with fields leaves the module in field mode with the fields that
// were added and the previous hash length (hasher_ is only rebuilt on
// success, hash_lb.cc:77-91).
#include <errno.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "module.h"

using bess::pb::Field;
using bess::pb::HashLBArg;
using bess::pb::HashLBCommandSetGatesArg;
using bess::pb::HashLBCommandSetModeArg;

class HashLB final : public Module {
 public:
  static const gate_idx_t kNumOGates = MAX_GATES;
  static constexpr size_t kMaxGates = 16384;  // hash_lb.h
  static const Commands kCmds;

  HashLB() : gates_(kMaxGates, 0) {}
  ~HashLB() override { bg_hlb_destroy(h_); }

  const Commands &cmds() const override { return kCmds; }

  // hash_lb.cc:115-134
  CommandResponse Init(const HashLBArg &arg) {
    int rc = bg_hlb_create(BG_HLB_L4, nullptr, 0, &h_);
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    HashLBCommandSetGatesArg gates_arg;
    for (int64_t g : arg.gates()) gates_arg.mutable_gates()->Add(g);
    CommandResponse ret = CommandSetGates(gates_arg);
    if (ret.code() != 0) return ret;
    if (arg.mode().empty() && !arg.fields_size()) {
      mode_ = BG_HLB_L4;  // kDefaultMode
      return Push();
    }
    HashLBCommandSetModeArg mode_arg;
    mode_arg.set_mode(arg.mode());
    for (const Field &f : arg.fields()) *mode_arg.add_fields() = f;
    return CommandSetMode(mode_arg);
  }

  // hash_lb.cc:76-98
  CommandResponse CommandSetMode(const HashLBCommandSetModeArg &arg) {
    if (arg.fields_size()) {
      mode_ = BG_HLB_FIELDS;
      fields_.clear();  // fields_table_ = ExactMatchTable<int>()
      int pos = 0;
      for (int i = 0; i < arg.fields_size(); i++) {
        const Field &f = arg.fields(i);
        // ExactMatchTable::DoAddField (exact_match_table.h:391-443) with
        // mask 0 (all bits); attr_name fields read offset() == 0
        const char *err = nullptr;
        char buf[96];
        const int size = (int)f.num_bytes();
        if (i >= BG_MAX_FIELDS) {
          snprintf(buf, sizeof(buf), "idx %d is not in [0,%d)", i, BG_MAX_FIELDS);
          err = buf;
        } else if (size < 1 || size > 8) {
          snprintf(buf, sizeof(buf), "idx %d: 'size' must be in [1,%d]", i, 8);
          err = buf;
        } else if ((int)f.offset() < 0 || (int)f.offset() > 1024) {
          snprintf(buf, sizeof(buf), "idx %d: invalid 'offset'", i);
          err = buf;
        }
        if (err) {
          Push();  // the partial table and the old hash length stay
          return CommandFailure(EINVAL, "Error adding field %d: %s", i, err);
        }
        fields_.push_back(bg_field{(int)f.offset(), size, pos, -1, 0});
        pos += size;
      }
      hash_len_ = (uint32_t)(pos + 7) / 8 * 8;  // hasher_(total_key_size())
    } else if (arg.mode() == "l2") {
      mode_ = BG_HLB_L2;
    } else if (arg.mode() == "l3") {
      mode_ = BG_HLB_L3;
    } else if (arg.mode() == "l4") {
      mode_ = BG_HLB_L4;
    } else {
      return CommandFailure(EINVAL, "available LB modes: l2, l3, l4");
    }
    return Push();
  }

  // hash_lb.cc:100-113
  CommandResponse CommandSetGates(const HashLBCommandSetGatesArg &arg) {
    if ((size_t)arg.gates_size() > kMaxGates)
      return CommandFailure(EINVAL, "HashLB can have at most %zu ogates",
                            kMaxGates);
    for (int i = 0; i < arg.gates_size(); i++) {
      gates_[i] = (gate_idx_t)arg.gates(i);
      if (!(gates_[i] < MAX_GATES || gates_[i] == DROP_GATE)) {
        Push();  // entries before i stay written
        return CommandFailure(EINVAL, "Invalid ogate %d", gates_[i]);
      }
    }
    num_gates_ = (size_t)arg.gates_size();
    return Push();
  }

  // hash_lb.cc:136-138
  std::string GetDesc() const override {
    char buf[32];
    snprintf(buf, sizeof(buf), "%zu fields", fields_.size());
    return buf;
  }

  int ProcessDevice(const bg_ctx &, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    return bg_hlb_classify(h_, d_frames, stride, n, 0, d_ogates, stream);
  }

  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    bg_hlb_window(h_, lo, hi);
    if (mode_ != BG_HLB_FIELDS) *lo = 0;
    *writeback = false;
  }

  int ProcessDeviceWindow(const bg_ctx &, void *d_win, size_t wstride, size_t n,
                          int win_off, uint16_t *d_ogates, void *stream) override {
    return bg_hlb_classify(h_, d_win, wstride, n, win_off, d_ogates, stream);
  }

 private:
  // mirror the control state into the device datapath
  CommandResponse Push() {
    int rc;
    if (mode_ == BG_HLB_FIELDS)
      rc = bg_hlb_set_mode(h_, mode_, fields_.data(), (int)fields_.size(),
                           (int)hash_len_);
    else
      rc = bg_hlb_set_mode(h_, mode_, nullptr, 0, -1);
    // gates_[0] is read when num_gates_ == 0 (hash_range(h, 0) == 0)
    if (rc == 0)
      rc = bg_hlb_set_gates(h_, gates_.data(), num_gates_ ? num_gates_ : 1,
                            num_gates_);
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    return CommandSuccess();
  }

  bg_hlb *h_ = nullptr;
  int mode_ = BG_HLB_L4;
  std::vector<bg_field> fields_;
  uint32_t hash_len_ = 0;  // hasher_(0) until a field set succeeds
  std::vector<gate_idx_t> gates_;
  size_t num_gates_ = 0;
};

const Commands HashLB::kCmds = {
    {"set_mode", "HashLBCommandSetModeArg",
     MODULE_CMD_FUNC(&HashLB::CommandSetMode), Command::THREAD_UNSAFE},
    {"set_gates", "HashLBCommandSetGatesArg",
     MODULE_CMD_FUNC(&HashLB::CommandSetGates), Command::THREAD_UNSAFE}};

ADD_MODULE_ARG(HashLB, bess::pb::HashLBArg, "hash_lb",
               "splits packets on a flow basis with L2/L3/L4 header fields")
