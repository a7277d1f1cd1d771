// bg_ttl_api.cc -- C ABI of the UpdateTTL datapath (include/bessgpu.h
// bg_update_ttl): no state, in place on a device frame slab.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include "bg_internal.h"

using namespace bg;

extern "C" int bg_update_ttl(int device, void *d_frames, size_t stride,
                             size_t n, uint16_t *d_out, bg_stream_t stream) {
  if (stride % 16 || stride < 32 || ((uintptr_t)d_frames & 15))
    return fail(EINVAL, "frame slab must be 16-byte aligned, stride a 16-byte "
                "multiple >= 32");
  int r = set_device(device);
  if (r) return r;
  TtlArgs a;
  memset(&a, 0, sizeof(a));
  a.frames = static_cast<uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.out = d_out;
  HIP_TRY(launch_ttl(a, num_cus(device), (hipStream_t)stream));
  return 0;
}
