// bg_wm_jit.h -- run-time compiled WildcardMatch kernels (bg_wm_jit.cc).
#ifndef BESS_AMD_BG_WM_JIT_H_
#define BESS_AMD_BG_WM_JIT_H_

#include <hip/hip_runtime.h>

#include <memory>
#include <string>

#include "bg_kernels.h"

namespace bg {

struct WmJit;
// The run-time compiled kernels for an image's tuple data (a) and the key
// plan of its fields at frame offset 0; shared by every image of the same
// shape, compiled on a background thread for `device`'s architecture.
// nullptr: no tag-word image.
std::shared_ptr<WmJit> wm_jit_request(const WmArgs &a, const FieldPlan &plan, uint32_t kw,
                                      int device);
// 1 ready, 0 compiling, -1 failed or none
int wm_jit_state(const WmJit *j);
// block until compiled (0), failed (-ENOEXEC) or timeout_ms passed (-ETIMEDOUT)
int wm_jit_wait(WmJit *j, int timeout_ms);
// Launch a's classification with the compiled kernel when it is ready and
// serves a (same plan, a tag-word image, paths allow it): true with *err
// the launch status; false when the caller must launch launch_wm.
bool wm_jit_launch(WmJit *j, const WmArgs &a, int device, int num_cus, hipStream_t s,
                   hipError_t *err);
std::string wm_jit_source(const WmJit *j);
// stop the compiler thread after the compile in progress (bg_shutdown)
void jit_shutdown();
// the generated source for a / plan (empty: no tag-word image)
std::string wm_jit_gen(const WmArgs &a, const FieldPlan &plan, uint32_t kw);
// compile a's source synchronously on the calling thread (no device needed):
// bg_wm_jit_check
int wm_jit_compile_now(const WmArgs &a, const FieldPlan &plan, uint32_t kw, std::string *log,
                       size_t *code_bytes);

}  // namespace bg

#endif  // BESS_AMD_BG_WM_JIT_H_
