"""NAT (core/modules/nat.{h,cc}): dynamic address/port translation. The
oracle restates Init, CreateNewEntry (port search from the module's Random,
eviction of expired mappings), ExtractEndpoint and Stamp; the GPU datapath
(bg_dnat: device lookup + rewrite, new mappings decided on the host in
packet order) must leave every packet byte and gate equal to the oracle's,
batch after batch: new flows, established flows (the device-only path),
reverse traffic, ICMP queries, protocols NAT drops, port 0, ports below
1024, suspended and exhausted ranges, and expiry after 300 s. The
reference seeds its Random from rdtsc; both sides take the same seed."""
import errno

import numpy as np
import pytest

from oracle import oracle as O
from oracle import oracle_more as OM

EXT = [{"ext_addr": "10.9.0.2", "port_ranges": [
           {"begin": 2000, "end": 2100},
           {"begin": 100, "end": 200, "suspended": True},
           {"begin": 5, "end": 900}]},
       {"ext_addr": "10.9.0.1"},
       {"ext_addr": "8.8.8.8", "port_ranges": [{"begin": 1024, "end": 1040}]}]
STRIDE = 128
T0 = 10**12


def flows(n, rng):
    """internal endpoints: (src ip, port, proto, icmp type)"""
    src = (0xC0A80000 | rng.integers(0, 1 << 16, n)).astype(np.uint64)
    r = rng.random(n)
    proto = np.where(r < 0.45, 6, np.where(r < 0.85, 17, np.where(r < 0.95, 1, 47)))
    port = rng.integers(1024, 65536, n)
    low = rng.random(n) < 0.15
    port[low] = rng.integers(1, 1024, int(low.sum()))
    port[rng.random(n) < 0.02] = 0
    itype = rng.choice([0, 8, 13, 15, 16, 3, 11], n)
    return src, port, proto, itype


def frames(src, sport, dst, dport, proto, itype, rng, ihl=None, stride=STRIDE):
    """Eth / IPv4 (IHL 5..7) / TCP, UDP or ICMP; valid checksums. In 64-byte
    slots the L4 payload is empty, so every frame fits its slot."""
    n = len(src)
    f = np.zeros((n, stride), np.uint8)
    extra = 16 if stride > 64 else 0
    f[:, 12:14] = [0x08, 0x00]
    if ihl is None:
        ihl = np.where(rng.random(n) < 0.8, 5, rng.integers(6, 8, n))
    f[:, 14] = 0x40 | ihl
    l4 = 14 + 4 * ihl
    for i in range(n):
        o = 14 + 20
        f[i, o:l4[i]] = rng.integers(0, 256, l4[i] - o)  # options
        pl = {6: 20, 17: 8, 1: 8}.get(int(proto[i]), 8) + extra
        iplen = 4 * ihl[i] + pl
        f[i, 16:18] = [iplen >> 8, iplen & 255]
        f[i, 18:20] = rng.integers(0, 256, 2)
        f[i, 22] = 64
        f[i, 23] = proto[i]
        f[i, 26:30] = np.frombuffer(int(src[i]).to_bytes(4, "big"), np.uint8)
        f[i, 30:34] = np.frombuffer(int(dst[i]).to_bytes(4, "big"), np.uint8)
        L = l4[i]
        f[i, L + 8:L + pl] = rng.integers(0, 256, pl - 8)
        if proto[i] in (6, 17):
            f[i, L:L + 2] = [sport[i] >> 8, sport[i] & 255]
            f[i, L + 2:L + 4] = [dport[i] >> 8, dport[i] & 255]
            if proto[i] == 17:
                f[i, L + 4:L + 6] = [pl >> 8, pl & 255]
            else:
                f[i, L + 12] = 0x50
        elif proto[i] == 1:
            f[i, L] = itype[i]
            f[i, L + 2:L + 4] = rng.integers(0, 256, 2)  # checksum: any
            f[i, L + 4:L + 6] = [sport[i] >> 8, sport[i] & 255]  # ident
    O.cksum_process(f, stride, n, 3, False)
    udp0 = np.nonzero((proto == 17) & (rng.random(n) < 0.1))[0]
    for i in udp0:  # UDP checksum 0: left alone
        f[i, l4[i] + 6:l4[i] + 8] = 0
    return f


def ext_side(g):
    """(addr, port) NAT gave each forwarded packet (its new source)"""
    ihl = g[:, 14] & 15
    l4 = 14 + 4 * ihl
    addr = np.array([int.from_bytes(g[i, 26:30].tobytes(), "big") for i in range(len(g))])
    port = np.array([int.from_bytes(g[i, l4[i]:l4[i] + 2].tobytes(), "big")
                     if g[i, 23] in (6, 17) else
                     int.from_bytes(g[i, l4[i] + 4:l4[i] + 6].tobytes(), "big")
                     for i in range(len(g))])
    return addr, port


def test_init_errors_match_oracle():
    from bess_amd.modules import NAT, ModuleError
    bad = [[{"ext_addr": "1.2.3.4", "port_ranges": [{"begin": 5, "end": 5}]}],
           [{"ext_addr": "1.2.3.4", "port_ranges": [{"begin": 5, "end": 70000}]}],
           [{"ext_addr": "1.2.3"}],
           [{"ext_addr": "bad", "port_ranges": [{"begin": 9, "end": 5}]}],
           []]
    for arg in bad:
        with pytest.raises(OM.OracleError) as eo:
            OM.OracleNAT(ext_addrs=arg)
        with pytest.raises(ModuleError) as em:
            NAT(ext_addrs=arg)
        assert em.value.code == eo.value.code == errno.EINVAL
        assert em.value.errmsg == eo.value.msg
    assert NAT(ext_addrs=EXT).desc() == OM.OracleNAT(ext_addrs=EXT).desc() == "0 entries"


def test_oracle_translation_keeps_checksums_valid():
    """Stamp's incremental updates leave valid IPv4 and TCP/UDP checksums
    (the reference's pin for incremental updates, checksum_test.cc:408-457)"""
    rng = np.random.default_rng(1)
    s, p, pr, it = flows(2000, rng)
    pr[:] = np.where(pr == 6, 6, 17)
    p[p == 0] = 4000
    f = frames(s, p, np.full(2000, 0x08080404), rng.integers(1, 65536, 2000), pr, it,
               rng, ihl=np.full(2000, 5))
    o = OM.OracleNAT(ext_addrs=EXT, seed=7)
    g = f.copy()
    out = o.process(g, STRIDE, 2000, 0, T0)
    ok = out == 1
    assert ok.sum() > 500  # the small ranges run out (drops)
    ipg, l4g = O.cksum_process(g, STRIDE, 2000, 3, True)
    assert (ipg[ok] == 0).all() and (l4g[ok] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("stride,ihl_mode", [(STRIDE, "mixed"), (64, "mixed"), (64, "ihl5")])
def test_gpu_batches_vs_oracle(stride, ihl_mode):
    """stride 64 runs the slab kernel (dnat_fused_slab_kernel); batches
    where no mapping can expire take the fused path (new flows listed and
    walked on the host, mixed with hits), the batch 301 s later the
    classify-then-decide path. ihl_mode "mixed": 20 % of frames carry IP
    options (IHL 6-7), so nearly every 64-packet tile has one; "ihl5": IHL 5
    everywhere but one packet in every seventh tile (a tile-uniform fast
    path for option-free headers was measured, scripts/ab/nat_reg_slot.py,
    and would be told apart by exactly this mix)"""
    import torch
    from bess_amd.modules import NAT
    rng = np.random.default_rng(11)
    m, o = NAT(ext_addrs=EXT, seed=0xABC), OM.OracleNAT(ext_addrs=EXT, seed=0xABC)

    def frames_(*fa, **kw):
        ihl = None
        if ihl_mode == "ihl5":
            ihl = np.full(len(fa[0]), 5)
            ihl[np.arange(len(ihl)) % 448 == 3] = 6
        return frames(*fa, ihl=ihl, stride=stride, **kw)

    def run(f, igate, now):
        ref = f.copy()
        want = o.process(ref, stride, len(f), igate, now)
        d = torch.from_numpy(f.reshape(-1).copy()).cuda()
        og = torch.zeros(len(f), dtype=torch.int16, device="cuda")
        m.process_device(d, stride, len(f), og, now, igate=igate)
        got = d.cpu().numpy().reshape(len(f), stride)
        assert (og.cpu().numpy().view(np.uint16) == want).all()
        bad = np.nonzero((got != ref).any(1))[0]
        assert len(bad) == 0, bad[:5]
        assert m.desc() == o.desc()
        return ref, want

    n = 6000
    s, p, pr, it = flows(1500, rng)
    pick = rng.integers(0, 1500, n)
    dst = rng.integers(1, 1 << 32, n)
    dport = rng.integers(1, 65536, n)
    fa = frames_(s[pick], p[pick], dst, dport, pr[pick], it[pick], rng)
    ga, out_a = run(fa, 0, T0)                            # new flows (host walk)
    mapped = out_a == 1
    assert 0.5 < mapped.mean() < 1.0 and int(m.desc().split()[0]) > 500
    run(fa[mapped], 0, T0 + 1000)                         # established: device only
    s3, p3, pr3, it3 = flows(800, rng)                    # hits mixed with new flows
    fc = frames_(s3, p3, rng.integers(1, 1 << 32, 800), rng.integers(1, 65536, 800),
                 pr3, it3, rng)
    mix = np.concatenate([fa[mapped][:1200], fc])
    run(mix[rng.permutation(len(mix))], 0, T0 + 1500)
    ea, ep = ext_side(ga[mapped])                         # reverse traffic
    k = int(mapped.sum())
    prm = pr[pick][mapped]
    # reverse endpoint: (dst, dst port) for TCP/UDP, (dst, ident) for ICMP
    rev = frames_(dst[mapped], np.where(prm == 1, ep, dport[mapped]), ea, ep, prm,
                 it[pick][mapped], rng)
    unk = frames_(rng.integers(1, 1 << 32, 500), rng.integers(1, 65536, 500),
                 rng.integers(1, 1 << 32, 500), rng.integers(1, 65536, 500),
                 np.full(500, 6), np.zeros(500, int), rng)
    run(np.concatenate([rev, unk]), 1, T0 + 2000)         # reverse hits + drops
    # 301 s later: new flows evict expired mappings where ports collide
    s2, p2, pr2, it2 = flows(3000, rng)
    fb = frames_(s2, p2, rng.integers(1, 1 << 32, 3000), rng.integers(1, 65536, 3000),
                pr2, it2, rng)
    run(fb, 0, T0 + 301 * 10**9)
    run(rev[:2000], 1, T0 + 302 * 10**9)                  # some mappings now gone


@pytest.mark.gpu
def test_gpu_ordered_after_default_stream_work(default_stream_backlog):
    """stream NULL is the caller's legacy default stream: the slab is
    written there behind a ~20 ms backlog right before the call, and NAT
    must translate those bytes, not the ones under them"""
    import torch
    from bess_amd.modules import NAT
    rng = np.random.default_rng(21)
    m, o = NAT(ext_addrs=EXT, seed=0x77), OM.OracleNAT(ext_addrs=EXT, seed=0x77)
    s, p, pr, it = flows(2000, rng)
    f = frames(s, p, rng.integers(1, 1 << 32, 2000), rng.integers(1, 65536, 2000), pr, it, rng)
    ref = f.copy()
    want = o.process(ref, STRIDE, len(f), 0, T0)
    d = torch.zeros(f.size, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(f.reshape(-1).copy()).cuda()
    og = torch.empty(len(f), dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    default_stream_backlog()
    d.copy_(src)
    og.fill_(0x1234)
    m.process_device(d, STRIDE, len(f), og, T0, igate=0)
    torch.cuda.synchronize()
    assert (og.cpu().numpy().view(np.uint16) == want).all()
    assert (d.cpu().numpy().reshape(len(f), STRIDE) == ref).all()


# ---- bessctl/module_tests/nat.py, restated (scapy is absent: packets are
# built field by field with scapy's defaults and fresh checksums)
def scapy_pkt(src, dst, kind, sport=0, dport=0, udp_ck0=False, icmp_id=0):
    import struct
    l7 = b"helloworld"
    if kind == "udp":
        l4 = struct.pack(">HHHH", sport, dport, 8 + len(l7), 0) + l7
        proto = 17
    elif kind == "tcp":  # seq 0, ack 0, dataofs 5, flags S, window 8192
        l4 = struct.pack(">HHIIBBHHH", sport, dport, 0, 0, 0x50, 0x02, 8192, 0, 0) + l7
        proto = 6
    else:                # echo-request, code 0, id, seq 0
        l4 = struct.pack(">BBHHH", 8, 0, 0, icmp_id, 0) + l7
        proto = 1
    ip = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + len(l4), 1, 0, 64, proto, 0,
                     bytes(int(x) for x in src.split(".")),
                     bytes(int(x) for x in dst.split(".")))
    eth = bytes.fromhex("06163e1b7232" "021e679f4dae" "0800")
    f = np.zeros((1, STRIDE), np.uint8)
    b = eth + ip + l4
    f[0, :len(b)] = np.frombuffer(b, np.uint8)
    O.cksum_process(f, STRIDE, 1, 3, False)  # IPv4 + TCP/UDP checksums
    if kind == "icmp":
        ck = O.lib().or_generic_checksum(f[0, 34:].ctypes.data, len(l4))
        f[0, 36:38] = [ck & 255, ck >> 8]
    if udp_ck0:
        f[0, 40:42] = 0
    return f, len(b)


CASES = [("udp", 56797, 53, False), ("udp", 56797, 53, True),
         ("tcp", 52428, 80, False), ("icmp", 0, 0, False)]


def module_test_case(kind, sport, dport, ck0, process):
    """nat.py _test_l4: orig -> natted (= a fresh packet from the rule
    address and the chosen port) -> reply -> unnatted (= the swapped
    original)"""
    f, ln = scapy_pkt("172.16.0.2", "8.8.8.8", kind, sport, dport, ck0)
    g = f.copy()
    assert list(process(g, 0)) == [1]
    l4 = 34
    chosen = int.from_bytes(g[0, l4 + (4 if kind == "icmp" else 0):][:2].tobytes(), "big")
    want, _ = scapy_pkt("192.168.1.1", "8.8.8.8", kind, chosen, dport, ck0, chosen)
    assert (g[0, :ln] == want[0, :ln]).all(), kind
    rep, _ = scapy_pkt("8.8.8.8", "192.168.1.1", kind, dport, chosen, ck0, chosen)
    assert list(process(rep, 1)) == [0]
    unn, _ = scapy_pkt("8.8.8.8", "172.16.0.2", kind, dport, sport, ck0, 0)
    assert (rep[0, :ln] == unn[0, :ln]).all(), kind


@pytest.mark.parametrize("case", CASES)
def test_oracle_vs_reference_module_test(case):
    o = OM.OracleNAT(ext_addrs=[{"ext_addr": "192.168.1.1"}], seed=3)
    module_test_case(*case, lambda f, g: o.process(f, STRIDE, 1, g, T0))


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_vs_reference_module_test(case):
    import torch
    from bess_amd.modules import NAT
    m = NAT(ext_addrs=[{"ext_addr": "192.168.1.1"}], seed=3)

    def process(f, igate):
        d = torch.from_numpy(f.reshape(-1).copy()).cuda()
        og = torch.zeros(1, dtype=torch.int16, device="cuda")
        m.process_device(d, STRIDE, 1, og, T0, igate=igate)
        f[:] = d.cpu().numpy().reshape(f.shape)
        return og.cpu().numpy().view(np.uint16)
    module_test_case(*case, process)


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["hit_first", "new_first", "interleaved"])
def test_gpu_expired_hits_in_order(order):
    """Every batch takes the fused pass: a forward hit on a
    mapping that has expired at `now` is not final -- a new flow earlier in
    the batch may evict it (CreateNewEntry, nat.cc:224-231), and a hit
    earlier in the batch refreshes it so that it can no longer be evicted
    (nat.cc:350-352) -- so such hits are listed and walked in packet order
    with the misses. Three external ports (3000..3002), three mappings of
    which two have idled past 300 s, and a new flow that must take a port."""
    import torch
    from bess_amd.modules import NAT
    ext = [{"ext_addr": "10.9.0.9", "port_ranges": [{"begin": 3000, "end": 3002}]}]
    rng = np.random.default_rng(5)
    for seed in range(6):
        m, o = NAT(ext_addrs=ext, seed=seed), OM.OracleNAT(ext_addrs=ext, seed=seed)
        src = np.array([0xC0A80001, 0xC0A80002, 0xC0A80003, 0xC0A80004], np.uint64)
        sport = np.array([4001, 4002, 4003, 4004])
        dst = np.full(4, 0x08080808, np.uint64)
        dport = np.full(4, 53)
        proto = np.full(4, 17)
        f = frames(src, sport, dst, dport, proto, np.zeros(4, int), rng,
                   ihl=np.full(4, 5))
        A, B, C, D = (f[i:i + 1] for i in range(4))

        def run(batch, now):
            ref = batch.copy()
            want = o.process(ref, STRIDE, len(batch), 0, now)
            d = torch.from_numpy(batch.reshape(-1).copy()).cuda()
            og = torch.zeros(len(batch), dtype=torch.int16, device="cuda")
            m.process_device(d, STRIDE, len(batch), og, now, igate=0)
            got = d.cpu().numpy().reshape(len(batch), STRIDE)
            assert (og.cpu().numpy().view(np.uint16) == want).all(), (order, seed)
            assert (got == ref).all(), (order, seed)
            return want

        assert list(run(np.concatenate([A, B, C]), T0)) == [1, 1, 1]
        run(A, T0 + 100 * 10**9)                      # A stays fresh
        now = T0 + 350 * 10**9                        # B and C have expired
        batch = {"hit_first": [B, D, C, B], "new_first": [D, B, C, B],
                 "interleaved": [C, D, B, A, D, C]}[order]
        run(np.concatenate(batch), now)
        run(np.concatenate([A, B, C, D]), now + 1)


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [STRIDE, 64])
def test_gpu_overlapping_internal_and_external_endpoints(stride):
    """The reference keeps both directions' entries in ONE map (nat.h), so
    when internal and external endpoints overlap: a reverse packet whose
    destination is an internal endpoint finds that forward entry and is
    translated with it; a forward packet whose source is an external
    endpoint finds its reverse entry; and a forward packet whose source
    endpoint an earlier packet of the same batch installs as an external
    endpoint meets the new entry. Sources here come from the NAT's own
    external addresses (10.9.0.1, 10.9.0.2, 8.8.8.8) as well as internal
    ones, batch after batch, every byte and gate as the oracle's."""
    import torch
    from bess_amd.modules import NAT
    rng = np.random.default_rng(23)
    ext = [{"ext_addr": "10.9.0.1", "port_ranges": [{"begin": 2000, "end": 2040}]},
           {"ext_addr": "10.9.0.2", "port_ranges": [{"begin": 2000, "end": 2040}]}]
    m, o = NAT(ext_addrs=ext, seed=0x77), OM.OracleNAT(ext_addrs=ext, seed=0x77)

    def run(f, igate, now):
        ref = f.copy()
        want = o.process(ref, stride, len(f), igate, now)
        d = torch.from_numpy(f.reshape(-1).copy()).cuda()
        og = torch.zeros(len(f), dtype=torch.int16, device="cuda")
        m.process_device(d, stride, len(f), og, now, igate=igate)
        got = d.cpu().numpy().reshape(len(f), stride)
        assert (og.cpu().numpy().view(np.uint16) == want).all()
        bad = np.nonzero((got != ref).any(1))[0]
        assert len(bad) == 0, bad[:5]
        return ref, want

    exts = np.array([0x0A090001, 0x0A090002], np.uint64)
    for b in range(4):
        n = 400
        internal = (0xC0A80000 | rng.integers(0, 64, n)).astype(np.uint64)
        use_ext = rng.random(n) < 0.4  # sources on the external side
        src = np.where(use_ext, exts[rng.integers(0, 2, n)], internal)
        sport = np.where(use_ext, rng.integers(2000, 2040, n), rng.integers(2000, 2040, n))
        proto = np.where(rng.random(n) < 0.5, 6, 17)
        dst = np.where(rng.random(n) < 0.5, exts[rng.integers(0, 2, n)],
                       (0xC0A80000 | rng.integers(0, 64, n)).astype(np.uint64))
        dport = rng.integers(2000, 2040, n)
        f = frames(src, sport, dst, dport, proto, np.zeros(n, int), rng,
                   ihl=np.full(n, 5), stride=stride)
        run(f, 0, T0 + b * 1000)
        # the same endpoints arriving on the external side: destinations
        # that are internal endpoints hit forward entries
        r = frames(dst, dport, src, sport, proto, np.zeros(n, int), rng,
                   ihl=np.full(n, 5), stride=stride)
        run(r, 1, T0 + b * 1000 + 500)
