// bg_rtc -- the run-time compiler of the WildcardMatch kernels specialised
// per rule-set shape (bg_wm_jit.cc), as a helper process next to
// libbessgpu.so.
//
// hiprtc runs the compiler library (LLVM) in the calling process. Inside a
// datapath process -- 16 worker threads launching kernels, the HIP runtime
// loading code objects -- that was not reliable: now and then a compile died
// (SIGSEGV inside hiprtcCompileProgram, once "LLVM ERROR: Cannot implicitly
// convert a scalable size ...") and took the whole process with it, and a
// process exiting mid-compile needed its exit ordered around the compiler's
// static destructors. Here a compile is its own process: it has no GPU, no
// other threads, and whatever happens to it, the library gets a status back
// and keeps launching the ahead-of-time kernel.
//
//   bg_rtc ARCH  < kernel source  > code object   (log on stderr)
// Exit status 0: compiled; 1: compile failed; 2: usage / I/O error.
#include <hip/hiprtc.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <string>

#include "bg_rtc_src.inc"  // kRtcNames / kRtcTexts (generated, rtc_embed.py)

static bool write_all(int fd, const char *p, size_t n) {
  while (n) {
    const ssize_t w = write(fd, p, n);
    if (w <= 0) return false;
    p += w;
    n -= (size_t)w;
  }
  return true;
}

int main(int argc, char **argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: bg_rtc ARCH < source > code\n");
    return 2;
  }
  std::string src;
  char buf[65536];
  for (;;) {
    const ssize_t r = read(0, buf, sizeof(buf));
    if (r < 0) return 2;
    if (r == 0) break;
    src.append(buf, (size_t)r);
  }
  hiprtcProgram prog;
  hiprtcResult r = hiprtcCreateProgram(&prog, src.c_str(), "bg_wm_jit.hip", kRtcHeaders,
                                       kRtcTexts, kRtcNames);
  if (r != HIPRTC_SUCCESS) {
    fprintf(stderr, "hiprtcCreateProgram: %s\n", hiprtcGetErrorString(r));
    return 1;
  }
  const std::string arch = std::string("--offload-arch=") + argv[1];
  const char *opts[] = {arch.c_str(), "-O3", "-std=c++17"};
  r = hiprtcCompileProgram(prog, 3, opts);
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  if (ls > 1) {
    std::string log(ls, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    (void)write_all(2, log.data(), strnlen(log.data(), log.size()));
  }
  int rc = 1;
  if (r == HIPRTC_SUCCESS) {
    size_t cs = 0;
    if (hiprtcGetCodeSize(prog, &cs) == HIPRTC_SUCCESS && cs) {
      std::string code(cs, '\0');
      if (hiprtcGetCode(prog, &code[0]) == HIPRTC_SUCCESS)
        rc = write_all(1, code.data(), code.size()) ? 0 : 2;
    }
  } else {
    fprintf(stderr, "hiprtcCompileProgram: %s\n", hiprtcGetErrorString(r));
  }
  hiprtcDestroyProgram(&prog);
  return rc;
}
