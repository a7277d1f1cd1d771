p='bess_amd/csrc/bg_kernels.hip'; s=open(p).read()
a="claim = min(max(kRingRunPackets / per, 1u), (uint32_t)kRingRunMax);"
assert s.count(a)==1; open(p,'w').write(s.replace(a, "claim = min(max(kRingRunPackets / per, 2u), (uint32_t)kRingRunMax);"))
