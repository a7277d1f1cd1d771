// bg_encap_api.cc -- C ABI of the IPEncap datapath (include/bessgpu.h
// bg_ip_encap): no state; packets in a device slab with per-packet head
// offsets and lengths (the mbuf's data_off / pkt_len), metadata in the slot.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include "bg_internal.h"

using namespace bg;

extern "C" int bg_ip_encap(int device, void *d_slots, size_t stride, size_t n,
                           int meta_off, const int32_t *attr_offsets,
                           uint16_t *d_head, uint32_t *d_len, uint16_t *d_out,
                           bg_stream_t stream) {
  if (!attr_offsets) return fail(EINVAL, "attr_offsets: 5 entries");
  if (meta_off < 0 || (size_t)meta_off >= stride)
    return fail(EINVAL, "meta_off %d outside the %zu-byte slot", meta_off, stride);
  static const int kSize[5] = {4, 4, 1, 4, 2};  // ip_encap.cc:36-40
  for (int i = 0; i < 5; i++)
    if (attr_offsets[i] >= 0 && (size_t)(meta_off + attr_offsets[i] + kSize[i]) > stride)
      return fail(EINVAL, "attribute %d at %d: past the slot", i, attr_offsets[i]);
  int r = set_device(device);
  if (r) return r;
  EncapArgs a;
  memset(&a, 0, sizeof(a));
  a.slots = static_cast<uint8_t *>(d_slots);
  a.stride = stride;
  a.n = n;
  a.meta_off = meta_off;
  for (int i = 0; i < 5; i++) a.offs[i] = attr_offsets[i];
  a.head = d_head;
  a.len = d_len;
  a.out = d_out;
  HIP_TRY(launch_encap(a, num_cus(device), (hipStream_t)stream));
  return 0;
}
