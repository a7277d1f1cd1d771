"""IPEncap (core/modules/ip_encap.cc:40-80): the oracle against a field-by-
field restatement of the header the module builds (the checksum checked
with the reference's own verify, checksum.h:211-228), prepend() failing
below 20 bytes of headroom (packet.h:145-154), invalid attribute offsets
(get_attr -> 0, set_attr skipped, core/module.h:686-705); the GPU kernel
bit-exact against the oracle on random slots: any head alignment, short
headrooms, invalid and overlapping attribute offsets."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import oracle_more as OM

STRIDE, META_OFF = 512, 448   # metadata area in the slot's last 64 bytes
OFFS = [(0, 4, 8, 12, 16),    # ip_src, ip_dst, ip_proto, ip_nexthop, ether_type
        (-1, 4, -2, 12, -1),  # invalid reads give 0, invalid writes skipped
        (20, 24, 30, 24, 26), # nexthop over ip_dst, ether_type over nexthop
        (60, 0, 63, -1, 62)]


def slots(n, seed):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, STRIDE), dtype=np.uint8)
    head = rng.integers(0, 300, n).astype(np.uint16)
    head[:8] = [0, 1, 19, 20, 21, 128, 131, 299]
    length = rng.integers(0, 65600, n).astype(np.uint32)  # total_len wraps
    return f, head, length


def test_oracle_header_fields():
    f, head, length = slots(200, 1)
    offs = OFFS[0]
    g, h, ln = f.copy(), head.copy(), length.copy()
    out = OM.ip_encap_process(g, STRIDE, 200, META_OFF, offs, h, ln)
    assert (out == 0).all()
    for i in range(200):
        meta = f[i, META_OFF:]
        if head[i] < 20:
            assert h[i] == head[i] and ln[i] == length[i]
            assert (g[i] == f[i]).all()
            continue
        nh = int(head[i]) - 20
        assert h[i] == nh and ln[i] == length[i] + 20
        ip = g[i, nh:nh + 20]
        tl = (int(length[i]) + 20) & 0xFFFF
        assert list(ip[:4]) == [0x45, 0, tl >> 8, tl & 255]
        assert list(ip[4:6]) == list(f[i, nh + 4:nh + 6])      # id untouched
        assert list(ip[6:10]) == [0x40, 0, 64, meta[offs[2]]]
        assert list(ip[12:16]) == list(meta[offs[0]:offs[0] + 4])
        assert list(ip[16:20]) == list(meta[offs[1]:offs[1] + 4])
        assert O.lib().or_ipv4_verify(ip.ctypes.data) == 1
        gm = g[i, META_OFF:]
        assert list(gm[offs[3]:offs[3] + 4]) == list(meta[offs[1]:offs[1] + 4])
        assert list(gm[offs[4]:offs[4] + 2]) == [8, 0]
        # nothing else in the slot changed
        mask = np.ones(STRIDE, bool)
        mask[nh:nh + 20] = False
        mask[META_OFF + offs[3]:META_OFF + offs[3] + 4] = False
        mask[META_OFF + offs[4]:META_OFF + offs[4] + 2] = False
        assert (g[i][mask] == f[i][mask]).all()


def test_oracle_invalid_offsets():
    f, head, length = slots(50, 2)
    head[:] = 100
    g, h, ln = f.copy(), head.copy(), length.copy()
    OM.ip_encap_process(g, STRIDE, 50, META_OFF, OFFS[1], h, ln)
    for i in range(50):
        ip = g[i, 80:100]
        assert list(ip[12:16]) == [0, 0, 0, 0] and ip[9] == 0   # src, proto
        assert list(ip[16:20]) == list(f[i, META_OFF + 4:META_OFF + 8])
        # ether_type (-1) never written; nexthop written
        assert list(g[i, META_OFF + 12:META_OFF + 16]) == list(ip[16:20])


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(OFFS)))
def test_gpu_vs_oracle(k):
    import torch
    from bess_amd.modules import IP_ENCAP_ATTRS, ip_encap
    n = 40000
    f, head, length = slots(n, 10 + k)
    ref, h, ln = f.copy(), head.copy(), length.copy()
    want = OM.ip_encap_process(ref, STRIDE, n, META_OFF, OFFS[k], h, ln)
    d = torch.from_numpy(f.reshape(-1)).cuda()
    dh = torch.from_numpy(head.view(np.int16)).cuda()
    dl = torch.from_numpy(length.view(np.int32)).cuda()
    og = torch.full((n,), -1, dtype=torch.int16, device="cuda")
    ip_encap(d, STRIDE, n, META_OFF,
             {a: o for a, o in zip(IP_ENCAP_ATTRS, OFFS[k]) if o >= 0}, dh, dl, og)
    assert (og.cpu().numpy().view(np.uint16) == want).all()
    assert (dh.cpu().numpy().view(np.uint16) == h).all()
    assert (dl.cpu().numpy().view(np.uint32) == ln).all()
    got = d.cpu().numpy().reshape(n, STRIDE)
    bad = np.nonzero((got != ref).any(1))[0]
    assert len(bad) == 0, bad[:5]
