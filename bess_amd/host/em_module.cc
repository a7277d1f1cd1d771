// em_module.cc -- ExactMatch: the reference module's control surface
// (core/modules/exact_match.{h,cc}, core/utils/exact_match_table.h) with the
// datapath on the GPU (bg_em_*, bg_kernels.hip em_classify_kernel).
//
// Same class name, commands table (names, argument types, thread safety),
// Init argument, error codes and messages and GetDesc as the reference; rule
// storage and lookups go through libbessgpu's device flow table.
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "../csrc/bg_internal.h"
#include "module.h"

namespace {

using bess::pb::EmptyArg;
using bess::pb::ExactMatchArg;
using bess::pb::ExactMatchCommandAddArg;
using bess::pb::ExactMatchCommandDeleteArg;
using bess::pb::ExactMatchCommandSetDefaultGateArg;
using bess::pb::ExactMatchConfig;
using bess::pb::Field;
using bess::pb::FieldData;

constexpr int kMaxFields = 8;     // MAX_FIELDS exact_match_table.h:50
constexpr int kMaxFieldSize = 8;  // MAX_FIELD_SIZE exact_match_table.h:51

bool valid_gate(gate_idx_t g) { return g < MAX_GATES || g == DROP_GATE; }

// endian.cc:36-58: value -> `size` bytes, big or little endian; false if
// the value does not fit
bool u64_to_bytes(uint8_t *out, uint64_t v, int size, bool big_endian) {
  for (int i = 0; i < size; i++) {
    out[big_endian ? size - 1 - i : i] = (uint8_t)(v & 0xFF);
    v >>= 8;
  }
  return v == 0;
}

// bess::utils::Copy of a value_bin into a u64 (memory order). The reference
// overruns the u64 for more than 8 bytes; that is rejected here.
bool bin_to_u64(const std::string &b, uint64_t *v) {
  if (b.size() > 8) return false;
  *v = 0;
  memcpy(v, b.data(), b.size());
  return true;
}

}  // namespace

class ExactMatch final : public Module {
 public:
  static const gate_idx_t kNumOGates = MAX_GATES;
  static const Commands kCmds;

  ~ExactMatch() override {
    rings_.clear();
    bg_em_destroy(table_);
  }

  const Commands &cmds() const override { return kCmds; }

  // exact_match.cc:93-119
  CommandResponse Init(const ExactMatchArg &arg) {
    empty_masks_ = arg.masks_size() == 0;
    if (arg.fields_size() != arg.masks_size() && !empty_masks_)
      return CommandFailure(EINVAL,
                            "must provide masks for all fields (or no masks for "
                            "default match on all bits on all fields)");
    for (int i = 0; i < arg.fields_size(); i++) {
      FieldData none;
      CommandResponse r =
          AddFieldOne(arg.fields(i), empty_masks_ ? none : arg.masks(i), i);
      if (r.code() != 0) return r;
    }
    default_gate_ = DROP_GATE;
    std::vector<bg_field> bf;
    for (size_t i = 0; i < num_fields_; i++) {
      const FieldSpec &f = fields_[i];
      bf.push_back(bg_field{f.offset, f.size, f.pos, f.attr_id, f.mask});
    }
    int rc = bg_em_create(bf.data(), (int)bf.size(), &table_);
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    return CommandSuccess();
  }

  // exact_match.cc:246-249
  std::string GetDesc() const override {
    char buf[64];
    snprintf(buf, sizeof(buf), "%zu fields, %zu rules", num_fields_,
             table_ ? bg_em_count(table_) : (size_t)0);
    return buf;
  }

  int ProcessDevice(const bg_ctx &c, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    int rc = bg_em_sync(table_, c.device, stream);
    if (rc < 0) return rc;
    return bg_em_classify(table_, d_frames, stride, n, default_gate_, d_ogates,
                          stream);
  }

  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    bg_em_window(table_, lo, hi);
    *writeback = false;
  }

  // P15: attr fields read the metadata area the slot carries at meta_off
  int BindMeta(int meta_off, const std::vector<std::string> &names,
               const std::vector<int32_t> &offsets) override {
    std::vector<int32_t> off = AttrOffsets(names, offsets);
    return bg_em_bind_meta(table_, meta_off, off.data(), (int)off.size());
  }

  int ProcessDeviceWindow(const bg_ctx &c, void *d_win, size_t wstride, size_t n,
                          int win_off, uint16_t *d_ogates, void *stream) override {
    int rc = bg_em_sync(table_, c.device, stream);
    if (rc < 0) return rc;
    return bg_em_classify_staged(table_, d_win, wstride, n, win_off, StagedMetaRow(),
                                 default_gate_, d_ogates, stream);
  }

  int MetaWindow(int *mlo, int *mhi) const override {
    return bg_em_meta_window(table_, mlo, mhi);
  }

  // the row offset of metadata byte 0 in a staged row (module.h StagedMetaAt)
  int StagedMetaRow() const {
    int lo, hi, mlo, mhi;
    bg_em_window(table_, &lo, &hi);
    if (bg_em_meta_window(table_, &mlo, &mhi) < 0 || mlo == mhi) return 0;
    return StagedMetaAt(lo, hi) - mlo;
  }

  // A pipe's slots go to one persistent classify kernel per device (bg_ring:
  // no HIP call per slot; the kernel reads the staged windows from pinned
  // host memory and writes the gates back there), re-created after a rule
  // change. Its workgroups take 2 per CU (half of each CU's LDS), leaving
  // room for other modules' kernels on the device.
  static const int kPipeRingLanes = 16;
  static const int kPipeRingRelease = 0;  // the done word: see PipeRingFor
  bool PipeRingCurrent(const PipeRing &ring, uint16_t *dflt) const override {
    if (ring.version != bg::em_version(table_) || ring.meta_row != StagedMetaRow()) return false;
    *dflt = default_gate_;
    return true;
  }
  int PipeRingFor(int device, std::shared_ptr<PipeRing> *out, uint16_t *dflt) override {
    out->reset();
    if (bg_get_path_flags() & BG_PATH_PIPE_NO_RING) return 0;
    int mlo, mhi;
    if (int rc = MetaWindow(&mlo, &mhi)) return rc;
    const int meta_row = StagedMetaRow();  // (attr fields: rows carry metadata)
    std::lock_guard<std::mutex> lk(ring_mu_);
    std::shared_ptr<PipeRing> &cur = rings_[device];
    if (!cur || cur->version != bg::em_version(table_) || cur->meta_row != meta_row) {
      int lo = 0, hi = 0;
      bg_em_window(table_, &lo, &hi);
      bg_ring *r = nullptr;
      const int rc = bg::em_ring_create(table_, device, kPipeRingLanes, 64,
                                        2 * bg::num_cus(device), 10000, lo,
                                        mlo == mhi ? bg::kSlabMeta : meta_row, &r);
      if (rc < 0) return rc;
      // per ticket: a system-scope acquire (measured as cheap as the CU's
      // L1 alone) and the done word stored once the gate stores -- system-
      // scope write-through stores into the pipe's uncached slots -- have
      // completed; a release there (an L2 write-back per ticket) halved the
      // 32-packet ticket rate (scripts/ring_coherence_ab.py)
      (void)bg_ring_set_coherence(r, 1, kPipeRingRelease);
      auto pr = std::make_shared<PipeRing>();
      pr->r = r;
      pr->meta_row = meta_row;
      pr->device = device;
      pr->lanes = kPipeRingLanes;
      pr->lane_mu.reset(new std::mutex[kPipeRingLanes]);
      pr->version = bg::ring_version(r);
      cur = std::move(pr);
    }
    *out = cur;
    *dflt = default_gate_;
    return 0;
  }

  // exact_match.cc:122-147
  CommandResponse GetInitialArg(const EmptyArg &) {
    ExactMatchArg r;
    for (size_t i = 0; i < num_fields_; i++) {
      const FieldSpec &f = fields_[i];
      Field *out = r.add_fields();
      if (f.attr_id >= 0)
        out->set_attr_name(all_attrs().at(f.attr_id).name);
      else
        out->set_offset((uint32_t)f.offset);
      out->set_num_bytes((uint32_t)f.size);
      if (!empty_masks_) r.add_masks()->set_value_bin(&f.mask, (size_t)f.size);
    }
    return CommandSuccess(r);
  }

  // exact_match.cc:150-187: rules sorted by gate, then field values
  CommandResponse GetRuntimeConfig(const EmptyArg &) {
    ExactMatchConfig r;
    r.set_default_gate(default_gate_);
    struct Rule {
      gate_idx_t gate;
      std::vector<std::string> vals;
    };
    std::vector<Rule> rules;
    size_t cur = 0;
    uint8_t key[BG_KEY_BYTES];
    uint16_t g;
    while (bg_em_iter(table_, &cur, key, &g)) {
      Rule rr;
      rr.gate = g;
      for (size_t i = 0; i < num_fields_; i++)
        rr.vals.emplace_back(reinterpret_cast<const char *>(key) + fields_[i].pos,
                             (size_t)fields_[i].size);
      rules.push_back(std::move(rr));
    }
    std::sort(rules.begin(), rules.end(), [](const Rule &a, const Rule &b) {
      if (a.gate != b.gate) return a.gate < b.gate;
      return a.vals < b.vals;
    });
    for (auto &rr : rules) {
      ExactMatchCommandAddArg *out = r.add_rules();
      out->set_gate(rr.gate);
      for (auto &v : rr.vals) out->add_fields()->set_value_bin(v.data(), v.size());
    }
    return CommandSuccess(r);
  }

  // exact_match.cc:210-222 (state may be partially restored on error)
  CommandResponse SetRuntimeConfig(const ExactMatchConfig &arg) {
    default_gate_ = (gate_idx_t)arg.default_gate();
    bg_em_clear(table_);
    for (int i = 0; i < arg.rules_size(); i++) {
      CommandResponse r = AddRule(arg.rules(i));
      if (r.code() != 0) return r;
    }
    return CommandSuccess();
  }

  CommandResponse CommandAdd(const ExactMatchCommandAddArg &arg) {
    return AddRule(arg);
  }

  // exact_match.cc:283-300
  CommandResponse CommandDelete(const ExactMatchCommandDeleteArg &arg) {
    if (arg.fields_size() == 0)
      return CommandFailure(EINVAL, "argument must be a list");
    uint8_t key[BG_KEY_BYTES];
    CommandResponse r = GatherKey(arg.fields(), key);
    if (r.code() != 0) return r;
    int rc = bg_em_delete(table_, key);
    if (rc < 0) return CommandFailure(-rc, "rule doesn't exist");
    return CommandSuccess();
  }

  CommandResponse CommandClear(const EmptyArg &) {
    bg_em_clear(table_);
    return CommandSuccess();
  }

  // exact_match.cc:307-311 (unvalidated, THREAD_SAFE)
  CommandResponse CommandSetDefaultGate(
      const ExactMatchCommandSetDefaultGateArg &arg) {
    default_gate_ = (gate_idx_t)arg.gate();
    return CommandSuccess();
  }

 private:
  struct FieldSpec {  // ExactMatchField (exact_match_table.h:126-140)
    uint64_t mask = 0;
    int attr_id = -1;
    int offset = 0;
    int pos = 0;
    int size = 0;
  };

  // AddFieldOne (exact_match.cc:62-91) + DoAddField (exact_match_table.h:
  // 391-443)
  CommandResponse AddFieldOne(const Field &field, const FieldData &mask,
                              int idx) {
    const int size = (int)field.num_bytes();
    uint64_t mask64 = 0;
    if (mask.encoding_case() == FieldData::kValueInt) {
      mask64 = mask.value_int();
    } else if (mask.encoding_case() == FieldData::kValueBin) {
      if (!bin_to_u64(mask.value_bin(), &mask64))
        return CommandFailure(EINVAL, "idx %d: not a valid %d-byte mask", idx,
                              size);
    }
    const bool is_attr = field.position_case() == Field::kAttrName;
    if (!is_attr && field.position_case() != Field::kOffset)
      return CommandFailure(EINVAL,
                            "idx %d: must specify 'offset' or 'attr_name'", idx);
    if (idx >= kMaxFields)
      return CommandFailure(EINVAL, "idx %d is not in [0,%d)", idx, kMaxFields);
    FieldSpec &f = fields_[idx];
    f.size = size;
    if (f.size < 1 || f.size > kMaxFieldSize)
      return CommandFailure(EINVAL, "idx %d: 'size' must be in [1,%d]", idx,
                            kMaxFieldSize);
    if (is_attr) {
      f.attr_id = AddMetadataAttr(field.attr_name(), (size_t)f.size);
      if (f.attr_id < 0)
        return CommandFailure(-f.attr_id, "idx %d: add_metadata_attr() failed",
                              idx);
      f.offset = 0;
    } else {
      f.attr_id = -1;
      f.offset = (int)field.offset();  // uint32 -> int
      if (f.offset < 0 || f.offset > 1024)
        return CommandFailure(EINVAL, "idx %d: invalid 'offset'", idx);
    }
    // offset fields take the mask big-endian, attribute fields host order
    const bool force_be = f.attr_id < 0;
    if (mask64 == 0) {
      // SetBitsHigh<uint64_t>(size * 8) -- the LOW size*8 bits (bits.h:180)
      f.mask = f.size >= 8 ? ~0ULL : ((1ULL << (8 * f.size)) - 1);
    } else {
      uint8_t b[8] = {0};
      if (!u64_to_bytes(b, mask64, f.size, force_be))
        return CommandFailure(EINVAL, "idx %d: not a valid %d-byte mask", idx,
                              f.size);
      f.mask = 0;
      memcpy(&f.mask, b, (size_t)f.size);
    }
    if (f.mask == 0) return CommandFailure(EINVAL, "idx %d: empty mask", idx);
    num_fields_++;
    f.pos = (int)raw_key_size_;
    raw_key_size_ += (size_t)f.size;
    return CommandSuccess();
  }

  // RuleFieldsFromPb (exact_match.cc:251-271) + gather_key
  // (exact_match_table.h:332-357)
  template <typename Rep>
  CommandResponse GatherKey(const Rep &vals, uint8_t *key) {
    const size_t n = (size_t)vals.size();
    std::vector<std::string> rule;
    for (size_t i = 0; i < n; i++) {
      const FieldData &v = vals.Get((int)i);
      const int fsize = i < (size_t)kMaxFields ? fields_[i].size : 0;
      if (v.encoding_case() == FieldData::kValueBin) {
        rule.push_back(v.value_bin());
      } else {  // value_int: little-endian, field size bytes
        uint64_t x = v.value_int();
        std::string s;
        for (int j = 0; j < fsize; j++) {
          s.push_back((char)(x & 0xFF));
          x >>= 8;
        }
        rule.push_back(s);
      }
    }
    if (n == 0) return CommandFailure(EINVAL, "rule has no fields");
    if (n != num_fields_)
      return CommandFailure(EINVAL, "rule should have %zu fields (has %zu)",
                            num_fields_, n);
    memset(key, 0, BG_KEY_BYTES);
    for (size_t i = 0; i < n; i++) {
      const FieldSpec &f = fields_[i];
      if ((size_t)f.size != rule[i].size())
        return CommandFailure(EINVAL,
                              "rule field %zu should have size %d (has %zu)", i,
                              f.size, rule[i].size());
      memcpy(key + f.pos, rule[i].data(), (size_t)f.size);
    }
    return CommandSuccess();
  }

  // AddRule (exact_match.cc:189-205 + exact_match_table.h:175-191)
  CommandResponse AddRule(const ExactMatchCommandAddArg &arg) {
    const gate_idx_t gate = (gate_idx_t)arg.gate();
    if (!valid_gate(gate)) return CommandFailure(EINVAL, "Invalid gate: %hu", gate);
    if (arg.fields_size() == 0)
      return CommandFailure(EINVAL, "'fields' must be a list");
    uint8_t key[BG_KEY_BYTES];
    CommandResponse r = GatherKey(arg.fields(), key);
    if (r.code() != 0) return r;
    int rc = bg_em_add(table_, key, gate);
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    return CommandSuccess();
  }

  FieldSpec fields_[kMaxFields];
  size_t num_fields_ = 0;
  size_t raw_key_size_ = 0;
  gate_idx_t default_gate_ = DROP_GATE;
  bool empty_masks_ = true;
  bg_em *table_ = nullptr;
  std::mutex ring_mu_;
  std::map<int, std::shared_ptr<PipeRing>> rings_;  // per device
};

// exact_match.cc:45-60
const Commands ExactMatch::kCmds = {
    {"get_initial_arg", "EmptyArg", MODULE_CMD_FUNC(&ExactMatch::GetInitialArg),
     Command::THREAD_SAFE},
    {"get_runtime_config", "EmptyArg",
     MODULE_CMD_FUNC(&ExactMatch::GetRuntimeConfig), Command::THREAD_SAFE},
    {"set_runtime_config", "ExactMatchConfig",
     MODULE_CMD_FUNC(&ExactMatch::SetRuntimeConfig), Command::THREAD_UNSAFE},
    {"add", "ExactMatchCommandAddArg", MODULE_CMD_FUNC(&ExactMatch::CommandAdd),
     Command::THREAD_UNSAFE},
    {"delete", "ExactMatchCommandDeleteArg",
     MODULE_CMD_FUNC(&ExactMatch::CommandDelete), Command::THREAD_UNSAFE},
    {"clear", "EmptyArg", MODULE_CMD_FUNC(&ExactMatch::CommandClear),
     Command::THREAD_UNSAFE},
    {"set_default_gate", "ExactMatchCommandSetDefaultGateArg",
     MODULE_CMD_FUNC(&ExactMatch::CommandSetDefaultGate), Command::THREAD_SAFE}};

ADD_MODULE_ARG(ExactMatch, ExactMatchArg, "em",
               "Multi-field classifier with an exact match table")
