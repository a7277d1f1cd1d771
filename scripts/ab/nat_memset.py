# NAT's per-call miss counter as before round 6's change: a memset node
# before each fused launch and the count read back into pageable memory
# (the product: two device words used in turn, pinned read-back)
import subprocess
src = subprocess.check_output(["git", "-C", "/root/repo", "show",
                               "fd4a592:bess_amd/csrc/bg_dnat_api.cc"]).decode()
open("bess_amd/csrc/bg_dnat_api.cc", "w").write(src)
