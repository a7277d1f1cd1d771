# Writing line ops (UpdateTTL, StaticNAT) on the slab writing back every slot
# of a tile, as before round 6 (the product writes back only the slots the
# op changed: profiles/r06/line_clean_ab_r06aq.json)
p = "bess_amd/csrc/bg_line_dev.h"
s = open(p).read()
a = """            ((dirty >> (u >> 2)) & 1))"""
assert s.count(a) == 1
s = s.replace(a, """            (dirty | 1))""")
open(p, "w").write(s)
