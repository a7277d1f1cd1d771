// wm_module.cc -- WildcardMatch: the reference module's control surface
// (core/modules/wildcard_match.{h,cc}) over libbessgpu's tuple-space tables
// (bg_wm_*, bg_kernels.hip wm_classify_kernel).
#include <inttypes.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "../csrc/bg_internal.h"
#include "module.h"

namespace {

using bess::pb::EmptyArg;
using bess::pb::Field;
using bess::pb::FieldData;
using bess::pb::WildcardMatchArg;
using bess::pb::WildcardMatchCommandAddArg;
using bess::pb::WildcardMatchCommandDeleteArg;
using bess::pb::WildcardMatchCommandSetDefaultGateArg;
using bess::pb::WildcardMatchConfig;

constexpr int kMaxFieldSize = 8;  // MAX_FIELD_SIZE wildcard_match.h:47

bool valid_gate(gate_idx_t g) { return g < MAX_GATES || g == DROP_GATE; }

}  // namespace

class WildcardMatch final : public Module {
 public:
  static const gate_idx_t kNumOGates = MAX_GATES;
  static const Commands kCmds;

  ~WildcardMatch() override {
    rings_.clear();
    bg_wm_destroy(table_);
  }

  const Commands &cmds() const override { return kCmds; }

  // wildcard_match.cc:111-134 (+ AddFieldOne 75-100)
  CommandResponse Init(const WildcardMatchArg &arg) {
    int size_acc = 0;
    for (int i = 0; i < arg.fields_size(); i++) {
      const Field &fd = arg.fields(i);
      fields_.emplace_back();
      WmField &f = fields_.back();
      f.pos = size_acc;
      f.size = (int)fd.num_bytes();
      if (f.size < 1 || f.size > kMaxFieldSize)
        return CommandFailure(EINVAL, "'size' must be 1-%d", kMaxFieldSize);
      if (fd.position_case() == Field::kOffset) {
        f.attr_id = -1;
        f.offset = (int)fd.offset();
        if (f.offset < 0 || f.offset > 1024)
          return CommandFailure(EINVAL, "too small 'offset'");
      } else if (fd.position_case() == Field::kAttrName) {
        f.attr_id = AddMetadataAttr(fd.attr_name(), (size_t)f.size);
        if (f.attr_id < 0)
          return CommandFailure(-f.attr_id, "add_metadata_attr() failed");
      } else {
        return CommandFailure(EINVAL, "specify 'offset' or 'attr'");
      }
      size_acc += f.size;
    }
    default_gate_ = DROP_GATE;
    total_key_size_ = (size_t)(size_acc + 7) / 8 * 8;
    std::vector<bg_field> bf;
    for (auto &f : fields_)
      bf.push_back(bg_field{f.offset, f.size, f.pos, f.attr_id, 0});
    int rc = bg_wm_create(bf.data(), (int)bf.size(), &table_);
    if (rc < 0) return CommandFailure(-rc, "%s", bg_last_error());
    return CommandSuccess();
  }

  // wildcard_match.cc:205-213
  std::string GetDesc() const override {
    size_t rules = 0;
    for (int t = 0; t < bg_wm_num_tuples(table_); t++)
      rules += bg_wm_tuple_count(table_, t);
    char buf[64];
    snprintf(buf, sizeof(buf), "%zu fields, %d rules", fields_.size(), (int)rules);
    return buf;
  }

  int ProcessDevice(const bg_ctx &c, void *d_frames, size_t stride, size_t n,
                    uint16_t *d_ogates, void *stream) override {
    int rc = bg_wm_sync(table_, c.device, stream);
    if (rc < 0) return rc;
    return bg_wm_classify(table_, d_frames, stride, n, default_gate_, d_ogates,
                          stream);
  }

  void DeviceWindow(int *lo, int *hi, bool *writeback) const override {
    bg_wm_window(table_, lo, hi);
    *writeback = false;
  }

  // P15: attr fields read the metadata area the slot carries at meta_off
  int BindMeta(int meta_off, const std::vector<std::string> &names,
               const std::vector<int32_t> &offsets) override {
    std::vector<int32_t> off = AttrOffsets(names, offsets);
    return bg_wm_bind_meta(table_, meta_off, off.data(), (int)off.size());
  }

  int ProcessDeviceWindow(const bg_ctx &c, void *d_win, size_t wstride, size_t n,
                          int win_off, uint16_t *d_ogates, void *stream) override {
    int rc = bg_wm_sync(table_, c.device, stream);
    if (rc < 0) return rc;
    return bg_wm_classify_staged(table_, d_win, wstride, n, win_off, StagedMetaRow(),
                                 default_gate_, d_ogates, stream);
  }

  int MetaWindow(int *mlo, int *mhi) const override {
    return bg_wm_meta_window(table_, mlo, mhi);
  }

  // As ExactMatch's: a pipe's slots go to one persistent classify kernel per
  // device (bg::wm_ring_create; the table probed in L2, no per-slot H2D /
  // launch / D2H), re-created after a rule change
  static const int kPipeRingLanes = 16;
  bool PipeRingCurrent(const PipeRing &ring, uint16_t *dflt) const override {
    if (ring.version != bg::wm_version(table_) || ring.meta_row != StagedMetaRow()) return false;
    *dflt = default_gate_;
    return true;
  }
  int PipeRingFor(int device, std::shared_ptr<PipeRing> *out, uint16_t *dflt) override {
    out->reset();
    if (bg_get_path_flags() & BG_PATH_PIPE_NO_RING) return 0;
    int mlo, mhi;
    if (int rc = MetaWindow(&mlo, &mhi)) return rc;
    const int meta_row = StagedMetaRow();
    std::lock_guard<std::mutex> lk(ring_mu_);
    std::shared_ptr<PipeRing> &cur = rings_[device];
    if (!cur || cur->version != bg::wm_version(table_) || cur->meta_row != meta_row) {
      int lo = 0, hi = 0;
      bg_wm_window(table_, &lo, &hi);
      bg_ring *r = nullptr;
      const int rc = bg::wm_ring_create(table_, device, kPipeRingLanes, 64,
                                        2 * bg::num_cus(device), 10000, lo,
                                        mlo == mhi ? bg::kSlabMeta : meta_row, &r);
      if (rc < 0) return rc;
      // per ticket a system-scope acquire, the done word relaxed (see
      // ExactMatch::PipeRingFor)
      (void)bg_ring_set_coherence(r, 1, 0);
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

  // the row offset of metadata byte 0 in a staged row (module.h StagedMetaAt)
  int StagedMetaRow() const {
    int lo, hi, mlo, mhi;
    bg_wm_window(table_, &lo, &hi);
    if (bg_wm_meta_window(table_, &mlo, &mhi) < 0 || mlo == mhi) return 0;
    return StagedMetaAt(lo, hi) - mlo;
  }

  // wildcard_match.cc:317-354
  CommandResponse CommandAdd(const WildcardMatchCommandAddArg &arg) {
    const gate_idx_t gate = (gate_idx_t)arg.gate();
    const int priority = (int)arg.priority();  // int64 -> int
    uint8_t key[BG_KEY_BYTES], mask[BG_KEY_BYTES];
    CommandResponse r = ExtractKeyMask(arg, key, mask);
    if (r.code() != 0) return r;
    if (!valid_gate(gate)) return CommandFailure(EINVAL, "Invalid gate: %hu", gate);
    int rc = bg_wm_add(table_, key, mask, priority, gate);
    if (rc == -ENOSPC)
      return CommandFailure(ENOSPC, "failed to add a new wildcard pattern");
    if (rc < 0) return CommandFailure(EINVAL, "failed to add a rule");
    return CommandSuccess();
  }

  // wildcard_match.cc:357-377
  CommandResponse CommandDelete(const WildcardMatchCommandDeleteArg &arg) {
    uint8_t key[BG_KEY_BYTES], mask[BG_KEY_BYTES];
    CommandResponse r = ExtractKeyMask(arg, key, mask);
    if (r.code() != 0) return r;
    int rc = bg_wm_delete(table_, key, mask);
    if (rc < 0) return CommandFailure(-rc, "failed to delete a rule");
    return CommandSuccess();
  }

  // wildcard_match.cc:379-388: tables emptied, tuples kept
  CommandResponse CommandClear(const EmptyArg &) {
    bg_wm_clear(table_);
    return CommandSuccess();
  }

  CommandResponse CommandSetDefaultGate(
      const WildcardMatchCommandSetDefaultGateArg &arg) {
    default_gate_ = (gate_idx_t)arg.gate();
    return CommandSuccess();
  }

  // wildcard_match.cc:391-405
  CommandResponse GetInitialArg(const EmptyArg &) {
    WildcardMatchArg r;
    for (auto &f : fields_) {
      Field *out = r.add_fields();
      if (f.attr_id >= 0)
        out->set_attr_name(all_attrs().at(f.attr_id).name);
      else
        out->set_offset((uint32_t)f.offset);
      out->set_num_bytes((uint32_t)f.size);
    }
    return CommandSuccess(r);
  }

  // wildcard_match.cc:409-460: sorted by priority, gate, masks, values
  CommandResponse GetRuntimeConfig(const EmptyArg &) {
    struct Rule {
      int32_t prio;
      gate_idx_t gate;
      std::vector<std::string> masks, vals;
    };
    std::vector<Rule> rules;
    for (int t = 0; t < bg_wm_num_tuples(table_); t++) {
      uint8_t mask[BG_KEY_BYTES], key[BG_KEY_BYTES];
      bg_wm_tuple_mask(table_, t, mask);
      size_t cur = 0;
      int32_t prio;
      uint16_t gate;
      while (bg_wm_iter(table_, t, &cur, key, &prio, &gate)) {
        Rule rr{prio, gate, {}, {}};
        for (auto &f : fields_) {
          rr.vals.emplace_back(reinterpret_cast<const char *>(key) + f.pos,
                               (size_t)f.size);
          rr.masks.emplace_back(reinterpret_cast<const char *>(mask) + f.pos,
                                (size_t)f.size);
        }
        rules.push_back(std::move(rr));
      }
    }
    std::sort(rules.begin(), rules.end(), [](const Rule &a, const Rule &b) {
      if (a.prio != b.prio) return a.prio < b.prio;
      if (a.gate != b.gate) return a.gate < b.gate;
      if (a.masks != b.masks) return a.masks < b.masks;
      return a.vals < b.vals;
    });
    WildcardMatchConfig r;
    r.set_default_gate(default_gate_);
    for (auto &rr : rules) {
      WildcardMatchCommandAddArg *out = r.add_rules();
      out->set_priority(rr.prio);
      out->set_gate(rr.gate);
      for (auto &v : rr.vals) out->add_values()->set_value_bin(v.data(), v.size());
      for (auto &m : rr.masks) out->add_masks()->set_value_bin(m.data(), m.size());
    }
    return CommandSuccess(r);
  }

  // wildcard_match.cc:469-481
  CommandResponse SetRuntimeConfig(const WildcardMatchConfig &arg) {
    bg_wm_clear(table_);
    default_gate_ = (gate_idx_t)arg.default_gate();
    for (int i = 0; i < arg.rules_size(); i++) {
      CommandResponse r = CommandAdd(arg.rules(i));
      if (r.code() != 0) return r;
    }
    return CommandSuccess();
  }

 private:
  struct WmField {  // wildcard_match.h:62-72
    int attr_id = -1;
    int offset = 0;
    int pos = 0;
    int size = 0;
  };

  // one FieldData -> u64 in key byte order (ExtractKeyMask 232-258)
  CommandResponse FieldValue(const FieldData &d, size_t i, int size,
                             const char *what, uint64_t *out) {
    *out = 0;
    if (d.encoding_case() == FieldData::kValueInt) {
      uint64_t v = d.value_int();
      uint8_t b[8] = {0};
      for (int j = 0; j < size; j++) {  // uint64_to_bin(..., true)
        b[size - 1 - j] = (uint8_t)(v & 0xFF);
        v >>= 8;
      }
      if (v)
        return CommandFailure(EINVAL, "idx %zu: not a correct %d-byte %s", i,
                              size, what);
      memcpy(out, b, (size_t)size);
    } else if (d.encoding_case() == FieldData::kValueBin) {
      const std::string &s = d.value_bin();
      if (s.size() > 8)  // the reference overruns a u64 here
        return CommandFailure(EINVAL, "idx %zu: not a correct %d-byte %s", i,
                              size, what);
      memcpy(out, s.data(), s.size());
    }
    return CommandSuccess();
  }

  template <typename T>
  CommandResponse ExtractKeyMask(const T &arg, uint8_t *key, uint8_t *mask) {
    if ((size_t)arg.values_size() != fields_.size())
      return CommandFailure(EINVAL, "must specify %zu values", fields_.size());
    if ((size_t)arg.masks_size() != fields_.size())
      return CommandFailure(EINVAL, "must specify %zu masks", fields_.size());
    memset(key, 0, BG_KEY_BYTES);
    memset(mask, 0, BG_KEY_BYTES);
    for (size_t i = 0; i < fields_.size(); i++) {
      const int size = fields_[i].size, pos = fields_[i].pos;
      uint64_t v, m;
      CommandResponse r = FieldValue(arg.values((int)i), i, size, "value", &v);
      if (r.code() != 0) return r;
      r = FieldValue(arg.masks((int)i), i, size, "mask", &m);
      if (r.code() != 0) return r;
      if (v & ~m)
        return CommandFailure(EINVAL,
                              "idx %zu: invalid pair of value 0x%0*" PRIx64
                              " and mask 0x%0*" PRIx64,
                              i, size * 2, v, size * 2, m);
      memcpy(key + pos, &v, (size_t)size);
      memcpy(mask + pos, &m, (size_t)size);
    }
    return CommandSuccess();
  }

  gate_idx_t default_gate_ = DROP_GATE;
  size_t total_key_size_ = 0;
  std::vector<WmField> fields_;
  bg_wm *table_ = nullptr;
  std::mutex ring_mu_;
  std::map<int, std::shared_ptr<PipeRing>> rings_;  // per device
};

// wildcard_match.cc:58-73
const Commands WildcardMatch::kCmds = {
    {"get_initial_arg", "EmptyArg",
     MODULE_CMD_FUNC(&WildcardMatch::GetInitialArg), Command::THREAD_SAFE},
    {"get_runtime_config", "EmptyArg",
     MODULE_CMD_FUNC(&WildcardMatch::GetRuntimeConfig), Command::THREAD_SAFE},
    {"set_runtime_config", "WildcardMatchConfig",
     MODULE_CMD_FUNC(&WildcardMatch::SetRuntimeConfig), Command::THREAD_UNSAFE},
    {"add", "WildcardMatchCommandAddArg",
     MODULE_CMD_FUNC(&WildcardMatch::CommandAdd), Command::THREAD_UNSAFE},
    {"delete", "WildcardMatchCommandDeleteArg",
     MODULE_CMD_FUNC(&WildcardMatch::CommandDelete), Command::THREAD_UNSAFE},
    {"clear", "EmptyArg", MODULE_CMD_FUNC(&WildcardMatch::CommandClear),
     Command::THREAD_UNSAFE},
    {"set_default_gate", "WildcardMatchCommandSetDefaultGateArg",
     MODULE_CMD_FUNC(&WildcardMatch::CommandSetDefaultGate),
     Command::THREAD_SAFE}};

ADD_MODULE_ARG(WildcardMatch, WildcardMatchArg, "wm",
               "Multi-field classifier with a wildcard match table")
