import os; exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'ring_noshare.py')).read())
p='bess_amd/csrc/bg_kernels.hip'; s=open(p).read()
a="""          if (nap < 4) {
            __builtin_amdgcn_s_sleep(2);
          } else if (nap < 8) {
            __builtin_amdgcn_s_sleep(8);
          } else {
            __builtin_amdgcn_s_sleep(32);
          }"""
b="""          __builtin_amdgcn_s_sleep(2);"""
assert s.count(a)==1; s=s.replace(a,b); open(p,'w').write(s)
