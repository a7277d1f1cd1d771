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

// Host packets (bessd's mbufs): slots[i] is packet i's slot (the buffer
// holding its metadata area at meta_off and its data at slots[i] +
// head[i]); slot_bytes of each are staged through the calling thread's
// pinned buffers, encapsulated on its stream, and copied back with the new
// head / len. Synchronous.
extern "C" int bg_ip_encap_host(int device, uint8_t *const *slots, size_t slot_bytes,
                                size_t n, int meta_off, const int32_t *attr_offsets,
                                uint16_t *head, uint32_t *len, uint16_t *out,
                                bg_stream_t stream) {
  if (n == 0) return 0;
  if (!slots || !head || !len || !out) return fail(EINVAL, "bad arguments");
  const size_t w = (slot_bytes + 15) / 16 * 16;
  for (size_t i = 0; i < n; i++)
    if ((size_t)head[i] + len[i] > slot_bytes)
      return fail(EINVAL, "packet %zu: data past the %zu-byte slot", i, slot_bytes);
  Staging &st = thread_staging();
  int r = set_device(device);
  if (r) return r;
  hipStream_t s = thread_stream(device, (hipStream_t)stream);
  // in: slots, then head (u16) and len (u32) arrays; out: gates
  const size_t arr = n * 8;
  r = st.ensure(device, n * w + arr, n * 2);
  if (r) return r;
  for (size_t i = 0; i < n; i++) {
    memcpy(st.h_in + i * w, slots[i], slot_bytes);
    if (w > slot_bytes) memset(st.h_in + i * w + slot_bytes, 0, w - slot_bytes);
  }
  uint16_t *hh = reinterpret_cast<uint16_t *>(st.h_in + n * w);
  uint32_t *hl = reinterpret_cast<uint32_t *>(st.h_in + n * w + n * 2 + (n & 1) * 2);
  memcpy(hh, head, n * 2);
  memcpy(hl, len, n * 4);
  const size_t total = n * w + arr;
  HIP_TRY(hipMemcpyAsync(st.d_in, st.h_in, total, hipMemcpyHostToDevice, s));
  uint16_t *dh = reinterpret_cast<uint16_t *>(st.d_in + n * w);
  uint32_t *dl = reinterpret_cast<uint32_t *>(st.d_in + n * w + n * 2 + (n & 1) * 2);
  r = bg_ip_encap(device, st.d_in, w, n, meta_off, attr_offsets, dh, dl,
                  reinterpret_cast<uint16_t *>(st.d_out), s);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(st.h_in, st.d_in, total, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(st.h_out, st.d_out, n * 2, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (size_t i = 0; i < n; i++) memcpy(slots[i], st.h_in + i * w, slot_bytes);
  memcpy(head, hh, n * 2);
  memcpy(len, hl, n * 4);
  memcpy(out, st.h_out, n * 2);
  return 0;
}
