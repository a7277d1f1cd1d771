# ACL's decision-tree slab op at ACL_OCC workgroups per CU (the product: 2;
# one measured 0.30 against 0.195 ms, profiles/r06/legs_ab_r06o.json, so the
# walk wants more waves): the launch still caps it at the occupancy limit
import os
occ = int(os.environ.get("ACL_OCC", "3"))
p = "bess_amd/csrc/bg_acl.hip"
s = open(p).read()
a = """struct AclTreeOp {
  using Args = AclArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 2;"""
assert s.count(a) == 1
s = s.replace(a, a.replace("kSlabPerCu = 2", "kSlabPerCu = %d" % occ))
open(p, "w").write(s)
