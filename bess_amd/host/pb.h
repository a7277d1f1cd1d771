// pb.h -- the protobuf messages of the classification path, with a
// hand-written proto3 wire codec (this image has no protoc / libprotobuf).
//
// Field numbers and types follow protobuf/module_msg.proto and
// protobuf/util_msg.proto of the reference (cited per message). Accessors
// use the names protoc would generate (fields_size(), fields(i),
// add_fields(), encoding_case(), value_bin(), ...) so module code reads the
// same against real generated headers.
#ifndef BESS_AMD_HOST_PB_H_
#define BESS_AMD_HOST_PB_H_

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace bess {
namespace pb {

// ---- wire helpers ------------------------------------------------------
class Reader {
 public:
  Reader(const void *p, size_t n)
      : p_(static_cast<const uint8_t *>(p)), end_(p_ + n) {}
  bool done() const { return p_ >= end_; }
  bool ok() const { return ok_; }
  // next field: number + wire type; false at end or on malformed input
  bool next(uint32_t *field, uint32_t *wt);
  bool varint(uint64_t *v);
  bool bytes(const uint8_t **d, size_t *n);
  bool skip(uint32_t wt);

 private:
  const uint8_t *p_, *end_;
  bool ok_ = true;
};

class Writer {
 public:
  void varint_field(uint32_t field, uint64_t v);
  void bytes_field(uint32_t field, const void *d, size_t n);
  void raw_varint(uint64_t v);
  std::string &str() { return s_; }

 private:
  std::string s_;
};

template <typename T>
class Repeated {
 public:
  int size() const { return (int)v_.size(); }
  const T &Get(int i) const { return v_[i]; }
  const T &operator[](int i) const { return v_[i]; }
  T *Add() {
    v_.emplace_back();
    return &v_.back();
  }
  T *Mutable(int i) { return &v_[i]; }
  typename std::vector<T>::iterator begin() { return v_.begin(); }
  typename std::vector<T>::iterator end() { return v_.end(); }
  typename std::vector<T>::const_iterator begin() const { return v_.begin(); }
  typename std::vector<T>::const_iterator end() const { return v_.end(); }
  void Clear() { v_.clear(); }

 private:
  std::vector<T> v_;
};

// Base of every message: parse/serialize entry points.
class Message {
 public:
  virtual ~Message() = default;
  bool ParseFromArray(const void *data, size_t n);
  std::string SerializeAsString() const;
  virtual bool MergeField(Reader &r, uint32_t field, uint32_t wt) = 0;
  virtual void Write(Writer &w) const = 0;
};

// util_msg.proto:45-50
class FieldData : public Message {
 public:
  enum EncodingCase { ENCODING_NOT_SET = 0, kValueBin = 1, kValueInt = 2 };
  EncodingCase encoding_case() const { return case_; }
  const std::string &value_bin() const { return bin_; }
  uint64_t value_int() const { return case_ == kValueInt ? int_ : 0; }
  void set_value_bin(const void *d, size_t n) {
    case_ = kValueBin;
    bin_.assign(static_cast<const char *>(d), n);
    int_ = 0;
  }
  void set_value_int(uint64_t v) {
    case_ = kValueInt;
    int_ = v;
    bin_.clear();
  }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  EncodingCase case_ = ENCODING_NOT_SET;
  std::string bin_;
  uint64_t int_ = 0;
};

// util_msg.proto:36-42
class Field : public Message {
 public:
  enum PositionCase { POSITION_NOT_SET = 0, kAttrName = 1, kOffset = 2 };
  PositionCase position_case() const { return case_; }
  const std::string &attr_name() const { return attr_; }
  uint32_t offset() const { return case_ == kOffset ? offset_ : 0; }
  uint32_t num_bytes() const { return num_bytes_; }
  void set_attr_name(const std::string &s) {
    case_ = kAttrName;
    attr_ = s;
    offset_ = 0;
  }
  void set_offset(uint32_t o) {
    case_ = kOffset;
    offset_ = o;
    attr_.clear();
  }
  void set_num_bytes(uint32_t n) { num_bytes_ = n; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  PositionCase case_ = POSITION_NOT_SET;
  std::string attr_;
  uint32_t offset_ = 0;
  uint32_t num_bytes_ = 0;
};

// module_msg.proto:50
class EmptyArg : public Message {
 public:
  bool MergeField(Reader &r, uint32_t, uint32_t wt) override {
    return r.skip(wt);
  }
  void Write(Writer &) const override {}
};

// module_msg.proto:501-504
class ExactMatchArg : public Message {
 public:
  int fields_size() const { return fields_.size(); }
  const Field &fields(int i) const { return fields_.Get(i); }
  Field *add_fields() { return fields_.Add(); }
  int masks_size() const { return masks_.size(); }
  const FieldData &masks(int i) const { return masks_.Get(i); }
  FieldData *add_masks() { return masks_.Add(); }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  Repeated<Field> fields_;
  Repeated<FieldData> masks_;
};

// module_msg.proto:69-72
class ExactMatchCommandAddArg : public Message {
 public:
  uint64_t gate() const { return gate_; }
  void set_gate(uint64_t g) { gate_ = g; }
  int fields_size() const { return fields_.size(); }
  const FieldData &fields(int i) const { return fields_.Get(i); }
  FieldData *add_fields() { return fields_.Add(); }
  const Repeated<FieldData> &fields() const { return fields_; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  uint64_t gate_ = 0;
  Repeated<FieldData> fields_;
};

// module_msg.proto:78-80
class ExactMatchCommandDeleteArg : public Message {
 public:
  int fields_size() const { return fields_.size(); }
  const FieldData &fields(int i) const { return fields_.Get(i); }
  FieldData *add_fields() { return fields_.Add(); }
  const Repeated<FieldData> &fields() const { return fields_; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  Repeated<FieldData> fields_;
};

// module_msg.proto:94-96 / 403-405: one `uint64 gate = 1`
class SetDefaultGateArg : public Message {
 public:
  uint64_t gate() const { return gate_; }
  void set_gate(uint64_t g) { gate_ = g; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  uint64_t gate_ = 0;
};
using ExactMatchCommandSetDefaultGateArg = SetDefaultGateArg;
using WildcardMatchCommandSetDefaultGateArg = SetDefaultGateArg;

// module_msg.proto:511-514
class ExactMatchConfig : public Message {
 public:
  uint64_t default_gate() const { return default_gate_; }
  void set_default_gate(uint64_t g) { default_gate_ = g; }
  int rules_size() const { return rules_.size(); }
  const ExactMatchCommandAddArg &rules(int i) const { return rules_.Get(i); }
  ExactMatchCommandAddArg *add_rules() { return rules_.Add(); }
  Repeated<ExactMatchCommandAddArg> *mutable_rules() { return &rules_; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  uint64_t default_gate_ = 0;
  Repeated<ExactMatchCommandAddArg> rules_;
};

// module_msg.proto:1152-1154
class WildcardMatchArg : public Message {
 public:
  int fields_size() const { return fields_.size(); }
  const Field &fields(int i) const { return fields_.Get(i); }
  Field *add_fields() { return fields_.Add(); }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  Repeated<Field> fields_;
};

// module_msg.proto:375-380
class WildcardMatchCommandAddArg : public Message {
 public:
  uint64_t gate() const { return gate_; }
  void set_gate(uint64_t g) { gate_ = g; }
  int64_t priority() const { return priority_; }
  void set_priority(int64_t p) { priority_ = p; }
  int values_size() const { return values_.size(); }
  const FieldData &values(int i) const { return values_.Get(i); }
  FieldData *add_values() { return values_.Add(); }
  int masks_size() const { return masks_.size(); }
  const FieldData &masks(int i) const { return masks_.Get(i); }
  FieldData *add_masks() { return masks_.Add(); }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  uint64_t gate_ = 0;
  int64_t priority_ = 0;
  Repeated<FieldData> values_;
  Repeated<FieldData> masks_;
};

// module_msg.proto:385-388
class WildcardMatchCommandDeleteArg : public Message {
 public:
  int values_size() const { return values_.size(); }
  const FieldData &values(int i) const { return values_.Get(i); }
  FieldData *add_values() { return values_.Add(); }
  int masks_size() const { return masks_.size(); }
  const FieldData &masks(int i) const { return masks_.Get(i); }
  FieldData *add_masks() { return masks_.Add(); }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  Repeated<FieldData> values_;
  Repeated<FieldData> masks_;
};

// module_msg.proto:1161-1164
class WildcardMatchConfig : public Message {
 public:
  uint64_t default_gate() const { return default_gate_; }
  void set_default_gate(uint64_t g) { default_gate_ = g; }
  int rules_size() const { return rules_.size(); }
  const WildcardMatchCommandAddArg &rules(int i) const { return rules_.Get(i); }
  WildcardMatchCommandAddArg *add_rules() { return rules_.Add(); }
  Repeated<WildcardMatchCommandAddArg> *mutable_rules() { return &rules_; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  uint64_t default_gate_ = 0;
  Repeated<WildcardMatchCommandAddArg> rules_;
};

// module_msg.proto:997-999 (IPChecksumArg) / 1010-1012 (L4ChecksumArg)
class VerifyArg : public Message {
 public:
  bool verify() const { return verify_; }
  void set_verify(bool v) { verify_ = v; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  bool verify_ = false;
};
using IPChecksumArg = VerifyArg;
using L4ChecksumArg = VerifyArg;

// ---- HashLB / ACL / IPLookup --------------------------------
// repeated int64 (proto3: packed on the wire; unpacked accepted too)
class Int64List {
 public:
  int size() const { return (int)v_.size(); }
  int64_t Get(int i) const { return v_[i]; }
  int64_t operator[](int i) const { return v_[i]; }
  void Add(int64_t x) { v_.push_back(x); }
  bool Merge(Reader &r, uint32_t wt);
  void Write(Writer &w, uint32_t field) const;
  typename std::vector<int64_t>::const_iterator begin() const { return v_.begin(); }
  typename std::vector<int64_t>::const_iterator end() const { return v_.end(); }

 private:
  std::vector<int64_t> v_;
};

// module_msg.proto:589-593
class HashLBArg : public Message {
 public:
  const Int64List &gates() const { return gates_; }
  Int64List *mutable_gates() { return &gates_; }
  const std::string &mode() const { return mode_; }
  void set_mode(const std::string &m) { mode_ = m; }
  int fields_size() const { return fields_.size(); }
  const Field &fields(int i) const { return fields_.Get(i); }
  Field *add_fields() { return fields_.Add(); }
  const Repeated<Field> &fields() const { return fields_; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  Int64List gates_;
  std::string mode_;
  Repeated<Field> fields_;
};

// module_msg.proto:116-119
class HashLBCommandSetModeArg : public Message {
 public:
  const std::string &mode() const { return mode_; }
  void set_mode(const std::string &m) { mode_ = m; }
  int fields_size() const { return fields_.size(); }
  const Field &fields(int i) const { return fields_.Get(i); }
  Field *add_fields() { return fields_.Add(); }
  Repeated<Field> *mutable_fields() { return &fields_; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  std::string mode_;
  Repeated<Field> fields_;
};

// module_msg.proto:126-128
class HashLBCommandSetGatesArg : public Message {
 public:
  const Int64List &gates() const { return gates_; }
  Int64List *mutable_gates() { return &gates_; }
  int gates_size() const { return gates_.size(); }
  int64_t gates(int i) const { return gates_.Get(i); }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  Int64List gates_;
};

// module_msg.proto:412-425
class ACLArg_Rule : public Message {
 public:
  const std::string &src_ip() const { return src_ip_; }
  const std::string &dst_ip() const { return dst_ip_; }
  uint32_t src_port() const { return src_port_; }
  uint32_t dst_port() const { return dst_port_; }
  bool established() const { return established_; }
  bool drop() const { return drop_; }
  void set_src_ip(const std::string &v) { src_ip_ = v; }
  void set_dst_ip(const std::string &v) { dst_ip_ = v; }
  void set_src_port(uint32_t v) { src_port_ = v; }
  void set_dst_port(uint32_t v) { dst_port_ = v; }
  void set_drop(bool v) { drop_ = v; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  std::string src_ip_, dst_ip_;
  uint32_t src_port_ = 0, dst_port_ = 0;
  bool established_ = false, drop_ = false;
};

class ACLArg : public Message {
 public:
  int rules_size() const { return rules_.size(); }
  const ACLArg_Rule &rules(int i) const { return rules_.Get(i); }
  const Repeated<ACLArg_Rule> &rules() const { return rules_; }
  ACLArg_Rule *add_rules() { return rules_.Add(); }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  Repeated<ACLArg_Rule> rules_;
};

// module_msg.proto:614-617
class IPLookupArg : public Message {
 public:
  uint32_t max_rules() const { return max_rules_; }
  uint32_t max_tbl8s() const { return max_tbl8s_; }
  void set_max_rules(uint32_t v) { max_rules_ = v; }
  void set_max_tbl8s(uint32_t v) { max_tbl8s_ = v; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  uint32_t max_rules_ = 0, max_tbl8s_ = 0;
};

// module_msg.proto:136-140 (gate unused by delete, 147-150)
class IPLookupCommandAddArg : public Message {
 public:
  const std::string &prefix() const { return prefix_; }
  uint64_t prefix_len() const { return prefix_len_; }
  uint64_t gate() const { return gate_; }
  void set_prefix(const std::string &v) { prefix_ = v; }
  void set_prefix_len(uint64_t v) { prefix_len_ = v; }
  void set_gate(uint64_t v) { gate_ = v; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  std::string prefix_;
  uint64_t prefix_len_ = 0, gate_ = 0;
};
using IPLookupCommandDeleteArg = IPLookupCommandAddArg;

using UpdateTTLArg = EmptyArg;

// module_msg.proto:729-741
class StaticNATArg_AddressRange : public Message {
 public:
  const std::string &start() const { return start_; }
  const std::string &end() const { return end_; }
  void set_start(const std::string &v) { start_ = v; }
  void set_end(const std::string &v) { end_ = v; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  std::string start_, end_;
};

class StaticNATArg_AddressRangePair : public Message {
 public:
  const StaticNATArg_AddressRange &int_range() const { return int_range_; }
  const StaticNATArg_AddressRange &ext_range() const { return ext_range_; }
  StaticNATArg_AddressRange *mutable_int_range() { return &int_range_; }
  StaticNATArg_AddressRange *mutable_ext_range() { return &ext_range_; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  StaticNATArg_AddressRange int_range_, ext_range_;
};

class StaticNATArg : public Message {
 public:
  int pairs_size() const { return pairs_.size(); }
  const StaticNATArg_AddressRangePair &pairs(int i) const { return pairs_.Get(i); }
  const Repeated<StaticNATArg_AddressRangePair> &pairs() const { return pairs_; }
  StaticNATArg_AddressRangePair *add_pairs() { return pairs_.Add(); }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  Repeated<StaticNATArg_AddressRangePair> pairs_;
};

// module_msg.proto:697-708
class NATArg_PortRange : public Message {
 public:
  uint32_t begin() const { return begin_; }
  uint32_t end() const { return end_; }
  bool suspended() const { return suspended_; }
  void set_begin(uint32_t v) { begin_ = v; }
  void set_end(uint32_t v) { end_ = v; }
  void set_suspended(bool v) { suspended_ = v; }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  uint32_t begin_ = 0, end_ = 0;
  bool suspended_ = false;
};

class NATArg_ExternalAddress : public Message {
 public:
  const std::string &ext_addr() const { return ext_addr_; }
  void set_ext_addr(const std::string &v) { ext_addr_ = v; }
  const Repeated<NATArg_PortRange> &port_ranges() const { return ranges_; }
  NATArg_PortRange *add_port_ranges() { return ranges_.Add(); }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  std::string ext_addr_;
  Repeated<NATArg_PortRange> ranges_;
};

class NATArg : public Message {
 public:
  const Repeated<NATArg_ExternalAddress> &ext_addrs() const { return addrs_; }
  NATArg_ExternalAddress *add_ext_addrs() { return addrs_.Add(); }
  bool MergeField(Reader &r, uint32_t field, uint32_t wt) override;
  void Write(Writer &w) const override;

 private:
  Repeated<NATArg_ExternalAddress> addrs_;
};

}  // namespace pb
}  // namespace bess

#endif  // BESS_AMD_HOST_PB_H_
