// TEST INFRASTRUCTURE ONLY. extern "C" entry into the reference's own
// core/utils/endian.cc (compiled unmodified from /root/reference by
// oracle/Makefile into oracle/_ref/, never committed, never shipped).
#include <cstddef>
#include <cstdint>

#include "endian.h"  // /root/reference/core/utils/endian.h

extern "C" int ref_uint64_to_bin(void *ptr, uint64_t val, size_t size,
                                 int big_endian) {
  return bess::utils::uint64_to_bin(ptr, val, size, big_endian != 0) ? 1 : 0;
}
