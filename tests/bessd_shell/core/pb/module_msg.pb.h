// Stand-in for the protoc-generated bess.pb messages the plugin wrappers
// name (tests only). A wrapper never looks inside a message: it forwards
// the serialized bytes to libbessgpu.so (bg_module_create / _command),
// which decodes them with its own proto3 codec; so each message here is
// its wire bytes, with protobuf's SerializeAsString / ParseFromArray /
// Any::PackFrom / UnpackTo names.
#ifndef BESSD_SHELL_MODULE_MSG_PB_H_
#define BESSD_SHELL_MODULE_MSG_PB_H_

#include <string>

namespace google {
namespace protobuf {

class Message {
 public:
  virtual ~Message() = default;
  std::string SerializeAsString() const { return bytes_; }
  bool ParseFromArray(const void *d, int n) {
    bytes_.assign(static_cast<const char *>(d), (size_t)n);
    return true;
  }
  bool ParseFromString(const std::string &s) {
    bytes_ = s;
    return true;
  }

 private:
  std::string bytes_;
};

class Any : public Message {
 public:
  void PackFrom(const Message &m) { ParseFromString(m.SerializeAsString()); }
  bool UnpackTo(Message *m) const { return m->ParseFromString(SerializeAsString()); }
};

}  // namespace protobuf
}  // namespace google

namespace bess {
namespace pb {

#define BESSD_SHELL_MSG(_N) \
  class _N : public google::protobuf::Message {};
BESSD_SHELL_MSG(EmptyArg)
BESSD_SHELL_MSG(ExactMatchArg)
BESSD_SHELL_MSG(ExactMatchConfig)
BESSD_SHELL_MSG(ExactMatchCommandAddArg)
BESSD_SHELL_MSG(ExactMatchCommandDeleteArg)
BESSD_SHELL_MSG(ExactMatchCommandSetDefaultGateArg)
BESSD_SHELL_MSG(WildcardMatchArg)
BESSD_SHELL_MSG(WildcardMatchConfig)
BESSD_SHELL_MSG(WildcardMatchCommandAddArg)
BESSD_SHELL_MSG(WildcardMatchCommandDeleteArg)
BESSD_SHELL_MSG(WildcardMatchCommandSetDefaultGateArg)
BESSD_SHELL_MSG(IPChecksumArg)
BESSD_SHELL_MSG(L4ChecksumArg)
BESSD_SHELL_MSG(HashLBArg)
BESSD_SHELL_MSG(HashLBCommandSetModeArg)
BESSD_SHELL_MSG(HashLBCommandSetGatesArg)
BESSD_SHELL_MSG(ACLArg)
BESSD_SHELL_MSG(IPLookupArg)
BESSD_SHELL_MSG(IPLookupCommandAddArg)
BESSD_SHELL_MSG(IPLookupCommandDeleteArg)
BESSD_SHELL_MSG(StaticNATArg)
BESSD_SHELL_MSG(NATArg)
BESSD_SHELL_MSG(IPEncapArg)
BESSD_SHELL_MSG(RewriteArg)
#undef BESSD_SHELL_MSG

}  // namespace pb
}  // namespace bess

#endif  // BESSD_SHELL_MODULE_MSG_PB_H_
