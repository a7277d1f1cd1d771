p='bess_amd/csrc/bg_kernels.h'; s=open(p).read()
a="constexpr uint32_t kRingRunPackets = kRingBlock * 4;"
assert s.count(a)==1; open(p,'w').write(s.replace(a, "constexpr uint32_t kRingRunPackets = kRingBlock * 16;"))
