# the LDS-table slab kernel (C2) at one workgroup per CU
p = 'bess_amd/csrc/bg_kernels.hip'
s = open(p).read()
a = """    if (a.t.lds == kLdsNone) pc = std::min(pc, 2);"""
b = """    if (a.t.lds == kLdsNone) pc = std::min(pc, 2);
    else pc = 1;"""
assert s.count(a) == 1
open(p, 'w').write(s.replace(a, b))
