# Hold sizes: LINE_HOLD sets line_kernel's kLineHold (bg_line_dev.h),
# LDS_HOLD em_slab_kernel's kGateHoldLds cap (bg_kernels.h).
import os
import re
for var, path, name in (("LINE_HOLD", "bess_amd/csrc/bg_line_dev.h", "kLineHold"),
                        ("LDS_HOLD", "bess_amd/csrc/bg_kernels.h", "kGateHoldLds")):
    if var in os.environ:
        s = open(path).read()
        s, k = re.subn(r"constexpr int %s = \d+;" % name,
                       "constexpr int %s = %s;" % (name, os.environ[var]), s)
        assert k == 1, name
        open(path, "w").write(s)
