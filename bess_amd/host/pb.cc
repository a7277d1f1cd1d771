// pb.cc -- proto3 wire codec for the messages in pb.h.
#include "pb.h"

namespace bess {
namespace pb {

enum : uint32_t { kVarint = 0, kFixed64 = 1, kLen = 2, kFixed32 = 5 };

bool Reader::varint(uint64_t *v) {
  uint64_t r = 0;
  for (int shift = 0; shift < 64 && p_ < end_; shift += 7) {
    uint8_t b = *p_++;
    r |= (uint64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) {
      *v = r;
      return true;
    }
  }
  ok_ = false;
  return false;
}

bool Reader::next(uint32_t *field, uint32_t *wt) {
  if (done()) return false;
  uint64_t tag;
  if (!varint(&tag)) return false;
  *field = (uint32_t)(tag >> 3);
  *wt = (uint32_t)(tag & 7);
  if (*field == 0) {
    ok_ = false;
    return false;
  }
  return true;
}

bool Reader::bytes(const uint8_t **d, size_t *n) {
  uint64_t len;
  if (!varint(&len)) return false;
  if (len > (uint64_t)(end_ - p_)) {
    ok_ = false;
    return false;
  }
  *d = p_;
  *n = (size_t)len;
  p_ += len;
  return true;
}

bool Reader::skip(uint32_t wt) {
  uint64_t v;
  const uint8_t *d;
  size_t n;
  switch (wt) {
    case kVarint: return varint(&v);
    case kFixed64:
      if (end_ - p_ < 8) return ok_ = false;
      p_ += 8;
      return true;
    case kLen: return bytes(&d, &n);
    case kFixed32:
      if (end_ - p_ < 4) return ok_ = false;
      p_ += 4;
      return true;
    default: return ok_ = false;
  }
}

void Writer::raw_varint(uint64_t v) {
  while (v >= 0x80) {
    s_.push_back((char)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  s_.push_back((char)v);
}

void Writer::varint_field(uint32_t field, uint64_t v) {
  raw_varint(((uint64_t)field << 3) | kVarint);
  raw_varint(v);
}

void Writer::bytes_field(uint32_t field, const void *d, size_t n) {
  raw_varint(((uint64_t)field << 3) | kLen);
  raw_varint(n);
  s_.append(static_cast<const char *>(d), n);
}

bool Message::ParseFromArray(const void *data, size_t n) {
  Reader r(data, n);
  uint32_t f, wt;
  while (r.next(&f, &wt))
    if (!MergeField(r, f, wt)) return false;
  return r.ok();
}

std::string Message::SerializeAsString() const {
  Writer w;
  Write(w);
  return w.str();
}

namespace {
bool read_u64(Reader &r, uint32_t wt, uint64_t *v) {
  if (wt != kVarint) return r.skip(wt);
  return r.varint(v);
}
template <typename M>
bool read_msg(Reader &r, uint32_t wt, M *m) {
  if (wt != kLen) return r.skip(wt);
  const uint8_t *d;
  size_t n;
  if (!r.bytes(&d, &n)) return false;
  return m->ParseFromArray(d, n);
}
template <typename M>
void write_msg(Writer &w, uint32_t field, const M &m) {
  std::string s = m.SerializeAsString();
  w.bytes_field(field, s.data(), s.size());
}
}  // namespace

// FieldData: bytes value_bin = 1; uint64 value_int = 2 (oneof)
bool FieldData::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1 && wt == kLen) {
    const uint8_t *d;
    size_t n;
    if (!r.bytes(&d, &n)) return false;
    set_value_bin(d, n);
    return true;
  }
  if (field == 2 && wt == kVarint) {
    uint64_t v;
    if (!r.varint(&v)) return false;
    set_value_int(v);
    return true;
  }
  return r.skip(wt);
}

void FieldData::Write(Writer &w) const {
  if (case_ == kValueBin) w.bytes_field(1, bin_.data(), bin_.size());
  if (case_ == kValueInt) w.varint_field(2, int_);
}

// Field: string attr_name = 1; uint32 offset = 2 (oneof); uint32 num_bytes = 3
bool Field::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  uint64_t v;
  if (field == 1 && wt == kLen) {
    const uint8_t *d;
    size_t n;
    if (!r.bytes(&d, &n)) return false;
    set_attr_name(std::string(reinterpret_cast<const char *>(d), n));
    return true;
  }
  if (field == 2 && wt == kVarint) {
    if (!r.varint(&v)) return false;
    set_offset((uint32_t)v);
    return true;
  }
  if (field == 3 && wt == kVarint) {
    if (!r.varint(&v)) return false;
    num_bytes_ = (uint32_t)v;
    return true;
  }
  return r.skip(wt);
}

void Field::Write(Writer &w) const {
  if (case_ == kAttrName) w.bytes_field(1, attr_.data(), attr_.size());
  if (case_ == kOffset) w.varint_field(2, offset_);
  if (num_bytes_) w.varint_field(3, num_bytes_);
}

bool ExactMatchArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_msg(r, wt, fields_.Add());
  if (field == 2) return read_msg(r, wt, masks_.Add());
  return r.skip(wt);
}
void ExactMatchArg::Write(Writer &w) const {
  for (auto &f : fields_) write_msg(w, 1, f);
  for (auto &m : masks_) write_msg(w, 2, m);
}

bool ExactMatchCommandAddArg::MergeField(Reader &r, uint32_t field,
                                         uint32_t wt) {
  if (field == 1) return read_u64(r, wt, &gate_);
  if (field == 2) return read_msg(r, wt, fields_.Add());
  return r.skip(wt);
}
void ExactMatchCommandAddArg::Write(Writer &w) const {
  if (gate_) w.varint_field(1, gate_);
  for (auto &f : fields_) write_msg(w, 2, f);
}

bool ExactMatchCommandDeleteArg::MergeField(Reader &r, uint32_t field,
                                            uint32_t wt) {
  if (field == 2) return read_msg(r, wt, fields_.Add());
  return r.skip(wt);
}
void ExactMatchCommandDeleteArg::Write(Writer &w) const {
  for (auto &f : fields_) write_msg(w, 2, f);
}

bool SetDefaultGateArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_u64(r, wt, &gate_);
  return r.skip(wt);
}
void SetDefaultGateArg::Write(Writer &w) const {
  if (gate_) w.varint_field(1, gate_);
}

bool ExactMatchConfig::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_u64(r, wt, &default_gate_);
  if (field == 2) return read_msg(r, wt, rules_.Add());
  return r.skip(wt);
}
void ExactMatchConfig::Write(Writer &w) const {
  if (default_gate_) w.varint_field(1, default_gate_);
  for (auto &x : rules_) write_msg(w, 2, x);
}

bool WildcardMatchArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_msg(r, wt, fields_.Add());
  return r.skip(wt);
}
void WildcardMatchArg::Write(Writer &w) const {
  for (auto &f : fields_) write_msg(w, 1, f);
}

bool WildcardMatchCommandAddArg::MergeField(Reader &r, uint32_t field,
                                            uint32_t wt) {
  uint64_t v;
  if (field == 1) return read_u64(r, wt, &gate_);
  if (field == 2) {
    if (wt != kVarint) return r.skip(wt);
    if (!r.varint(&v)) return false;
    priority_ = (int64_t)v;
    return true;
  }
  if (field == 3) return read_msg(r, wt, values_.Add());
  if (field == 4) return read_msg(r, wt, masks_.Add());
  return r.skip(wt);
}
void WildcardMatchCommandAddArg::Write(Writer &w) const {
  if (gate_) w.varint_field(1, gate_);
  if (priority_) w.varint_field(2, (uint64_t)priority_);
  for (auto &x : values_) write_msg(w, 3, x);
  for (auto &x : masks_) write_msg(w, 4, x);
}

bool WildcardMatchCommandDeleteArg::MergeField(Reader &r, uint32_t field,
                                               uint32_t wt) {
  if (field == 1) return read_msg(r, wt, values_.Add());
  if (field == 2) return read_msg(r, wt, masks_.Add());
  return r.skip(wt);
}
void WildcardMatchCommandDeleteArg::Write(Writer &w) const {
  for (auto &x : values_) write_msg(w, 1, x);
  for (auto &x : masks_) write_msg(w, 2, x);
}

bool WildcardMatchConfig::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_u64(r, wt, &default_gate_);
  if (field == 2) return read_msg(r, wt, rules_.Add());
  return r.skip(wt);
}
void WildcardMatchConfig::Write(Writer &w) const {
  if (default_gate_) w.varint_field(1, default_gate_);
  for (auto &x : rules_) write_msg(w, 2, x);
}

bool VerifyArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  uint64_t v;
  if (field == 1 && wt == kVarint) {
    if (!r.varint(&v)) return false;
    verify_ = v != 0;
    return true;
  }
  return r.skip(wt);
}
void VerifyArg::Write(Writer &w) const {
  if (verify_) w.varint_field(1, 1);
}

// ---- HashLB / ACL / IPLookup -------------------------------------------
namespace {
bool read_str(Reader &r, uint32_t wt, std::string *s) {
  if (wt != kLen) return r.skip(wt);
  const uint8_t *d;
  size_t n;
  if (!r.bytes(&d, &n)) return false;
  s->assign(reinterpret_cast<const char *>(d), n);
  return true;
}
bool read_bool(Reader &r, uint32_t wt, bool *b) {
  uint64_t v;
  if (wt != kVarint) return r.skip(wt);
  if (!r.varint(&v)) return false;
  *b = v != 0;
  return true;
}
bool read_u32(Reader &r, uint32_t wt, uint32_t *x) {
  uint64_t v;
  if (wt != kVarint) return r.skip(wt);
  if (!r.varint(&v)) return false;
  *x = (uint32_t)v;
  return true;
}
void write_str(Writer &w, uint32_t field, const std::string &s) {
  if (!s.empty()) w.bytes_field(field, s.data(), s.size());
}
}  // namespace

bool Int64List::Merge(Reader &r, uint32_t wt) {
  uint64_t v;
  if (wt == kVarint) {
    if (!r.varint(&v)) return false;
    v_.push_back((int64_t)v);
    return true;
  }
  if (wt != kLen) return r.skip(wt);
  const uint8_t *d;
  size_t n;
  if (!r.bytes(&d, &n)) return false;
  Reader sub(d, n);
  while (!sub.done()) {
    if (!sub.varint(&v)) return false;
    v_.push_back((int64_t)v);
  }
  return true;
}

void Int64List::Write(Writer &w, uint32_t field) const {
  if (v_.empty()) return;
  Writer packed;
  for (int64_t x : v_) packed.raw_varint((uint64_t)x);
  w.bytes_field(field, packed.str().data(), packed.str().size());
}

bool HashLBArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return gates_.Merge(r, wt);
  if (field == 2) return read_str(r, wt, &mode_);
  if (field == 3) return read_msg(r, wt, fields_.Add());
  return r.skip(wt);
}
void HashLBArg::Write(Writer &w) const {
  gates_.Write(w, 1);
  write_str(w, 2, mode_);
  for (auto &f : fields_) write_msg(w, 3, f);
}

bool HashLBCommandSetModeArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_str(r, wt, &mode_);
  if (field == 2) return read_msg(r, wt, fields_.Add());
  return r.skip(wt);
}
void HashLBCommandSetModeArg::Write(Writer &w) const {
  write_str(w, 1, mode_);
  for (auto &f : fields_) write_msg(w, 2, f);
}

bool HashLBCommandSetGatesArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return gates_.Merge(r, wt);
  return r.skip(wt);
}
void HashLBCommandSetGatesArg::Write(Writer &w) const { gates_.Write(w, 1); }

bool ACLArg_Rule::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  switch (field) {
    case 1: return read_str(r, wt, &src_ip_);
    case 2: return read_str(r, wt, &dst_ip_);
    case 3: return read_u32(r, wt, &src_port_);
    case 4: return read_u32(r, wt, &dst_port_);
    case 5: return read_bool(r, wt, &established_);
    case 6: return read_bool(r, wt, &drop_);
    default: return r.skip(wt);
  }
}
void ACLArg_Rule::Write(Writer &w) const {
  write_str(w, 1, src_ip_);
  write_str(w, 2, dst_ip_);
  if (src_port_) w.varint_field(3, src_port_);
  if (dst_port_) w.varint_field(4, dst_port_);
  if (established_) w.varint_field(5, 1);
  if (drop_) w.varint_field(6, 1);
}

bool ACLArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_msg(r, wt, rules_.Add());
  return r.skip(wt);
}
void ACLArg::Write(Writer &w) const {
  for (auto &x : rules_) write_msg(w, 1, x);
}

bool IPLookupArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_u32(r, wt, &max_rules_);
  if (field == 2) return read_u32(r, wt, &max_tbl8s_);
  return r.skip(wt);
}
void IPLookupArg::Write(Writer &w) const {
  if (max_rules_) w.varint_field(1, max_rules_);
  if (max_tbl8s_) w.varint_field(2, max_tbl8s_);
}

bool IPLookupCommandAddArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_str(r, wt, &prefix_);
  if (field == 2) return read_u64(r, wt, &prefix_len_);
  if (field == 3) return read_u64(r, wt, &gate_);
  return r.skip(wt);
}
void IPLookupCommandAddArg::Write(Writer &w) const {
  write_str(w, 1, prefix_);
  if (prefix_len_) w.varint_field(2, prefix_len_);
  if (gate_) w.varint_field(3, gate_);
}

bool StaticNATArg_AddressRange::MergeField(Reader &r, uint32_t field,
                                           uint32_t wt) {
  if (field == 1) return read_str(r, wt, &start_);
  if (field == 2) return read_str(r, wt, &end_);
  return r.skip(wt);
}
void StaticNATArg_AddressRange::Write(Writer &w) const {
  write_str(w, 1, start_);
  write_str(w, 2, end_);
}

bool StaticNATArg_AddressRangePair::MergeField(Reader &r, uint32_t field,
                                               uint32_t wt) {
  if (field == 1) return read_msg(r, wt, &int_range_);
  if (field == 2) return read_msg(r, wt, &ext_range_);
  return r.skip(wt);
}
void StaticNATArg_AddressRangePair::Write(Writer &w) const {
  write_msg(w, 1, int_range_);
  write_msg(w, 2, ext_range_);
}

bool StaticNATArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_msg(r, wt, pairs_.Add());
  return r.skip(wt);
}
void StaticNATArg::Write(Writer &w) const {
  for (auto &x : pairs_) write_msg(w, 1, x);
}

bool NATArg_PortRange::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_u32(r, wt, &begin_);
  if (field == 2) return read_u32(r, wt, &end_);
  if (field == 3) return read_bool(r, wt, &suspended_);
  return r.skip(wt);
}
void NATArg_PortRange::Write(Writer &w) const {
  if (begin_) w.varint_field(1, begin_);
  if (end_) w.varint_field(2, end_);
  if (suspended_) w.varint_field(3, 1);
}

bool NATArg_ExternalAddress::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_str(r, wt, &ext_addr_);
  if (field == 2) return read_msg(r, wt, ranges_.Add());
  return r.skip(wt);
}
void NATArg_ExternalAddress::Write(Writer &w) const {
  write_str(w, 1, ext_addr_);
  for (auto &x : ranges_) write_msg(w, 2, x);
}

bool NATArg::MergeField(Reader &r, uint32_t field, uint32_t wt) {
  if (field == 1) return read_msg(r, wt, addrs_.Add());
  return r.skip(wt);
}
void NATArg::Write(Writer &w) const {
  for (auto &x : addrs_) write_msg(w, 1, x);
}

}  // namespace pb
}  // namespace bess
