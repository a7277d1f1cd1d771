p='bess_amd/csrc/bg_kernels.hip'; s=open(p).read()
a="""        if (a.nlanes > 1) {
          const uint32_t cand = (home + wl) % a.nlanes;"""
b="""        if (false) {
          const uint32_t cand = (home + wl) % a.nlanes;"""
assert s.count(a)==1; s=s.replace(a,b); open(p,'w').write(s)
