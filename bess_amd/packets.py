"""Synthetic traffic and rule sets for the classification path.

The role of BESS's Source / Rewrite modules (core/modules/source.cc:40-101,
rewrite.cc:90-134) for benchmarks and parity tests: fixed-stride frame slabs
(frame i at byte i*stride, = Packet::head_data()) holding Eth / IPv4 (IHL 5) /
UDP or TCP headers. "S-byte packet" follows BESS's wire convention: the frame
is S-4 bytes (Source default pkt_size 60 = a 64 B packet, source.cc:47).

numpy only; the result is uploaded to HBM by the caller.
"""
import numpy as np

ETH_DST = bytes.fromhex("06163e1b7232")  # bessctl/conf/samples/exactmatch.bess
ETH_SRC = bytes.fromhex("021e679f4dae")

# 5-tuple fields, untagged Eth / IPv4 IHL=5: (offset, size)
FIVE_TUPLE = [(23, 1), (26, 4), (30, 4), (34, 2), (36, 2)]

IMIX = ((60, 7), (590, 4), (1514, 1))  # frame bytes : weight (64/594/1518 B)


def default_mask(size):
    """SetBitsHigh<uint64_t>(size*8) (bits.h:180-185): the low size*8 bits."""
    return (1 << (8 * size)) - 1 if size < 8 else (1 << 64) - 1


def em_fields_5tuple():
    """[(offset, size, mask)] as ExactMatchTable::AddField resolves a field
    given with mask 0 (exact_match_table.h:420-422)."""
    return [(o, s, default_mask(s)) for o, s in FIVE_TUPLE]


def random_tuples(n, rng, protos=(6, 17)):
    """n distinct 5-tuples as a dict of arrays."""
    out = {"proto": rng.choice(np.array(protos, np.uint8), n),
           "sip": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
           "dip": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
           "sport": rng.integers(0, 1 << 16, n).astype(np.uint16),
           "dport": rng.integers(0, 1 << 16, n).astype(np.uint16)}
    k = tuple_keys(out)
    _, first = np.unique(k.view("S16").ravel(), return_index=True)
    if len(first) != n:  # astronomically rare: redraw duplicates
        keep = np.sort(first)
        out = {f: v[keep] for f, v in out.items()}
        extra = random_tuples(n - len(keep), rng, protos)
        out = {f: np.concatenate([out[f], extra[f]]) for f in out}
    return out


def tuple_keys(t):
    """ExactMatch key bytes of 5-tuples: proto | sip | dip | sport | dport in
    wire order (13 bytes, zero padded to total_key_size = 16)."""
    n = len(t["proto"])
    k = np.zeros((n, 16), np.uint8)
    k[:, 0] = t["proto"]
    k[:, 1:5] = t["sip"].astype(">u4").view(np.uint8).reshape(n, 4)
    k[:, 5:9] = t["dip"].astype(">u4").view(np.uint8).reshape(n, 4)
    k[:, 9:11] = t["sport"].astype(">u2").view(np.uint8).reshape(n, 2)
    k[:, 11:13] = t["dport"].astype(">u2").view(np.uint8).reshape(n, 2)
    return k


def build_frames(t, frame_len, stride, rng=None, payload="zero", out=None,
                 ip_csum="zero"):
    """Eth/IPv4/{UDP,TCP} frames for tuples `t` into an (n, stride) uint8
    slab. UDP/TCP chosen by t['proto'] (6 -> TCP, else UDP header layout).
    Checksum fields are left 0 (or random with ip_csum='random')."""
    n = len(t["proto"])
    if isinstance(frame_len, (int, np.integer)):
        frame_len = np.full(n, frame_len, np.int64)
    frame_len = np.asarray(frame_len, np.int64)
    f = out if out is not None else np.zeros((n, stride), np.uint8)
    if payload == "random":
        rng = rng or np.random.default_rng(0)
        f.reshape(-1)[:] = np.frombuffer(rng.bytes(f.size), np.uint8)
        # zero the bytes past each frame so slabs are deterministic
        for L in np.unique(frame_len):
            if L < stride:
                f[frame_len == L, int(L):] = 0
    f[:, 0:6] = np.frombuffer(ETH_DST, np.uint8)
    f[:, 6:12] = np.frombuffer(ETH_SRC, np.uint8)
    f[:, 12] = 0x08
    f[:, 13] = 0x00
    f[:, 14] = 0x45
    f[:, 15] = 0
    ip_len = (frame_len - 14).astype(">u2")
    f[:, 16:18] = ip_len.view(np.uint8).reshape(n, 2)
    f[:, 18:20] = 0
    f[:, 20:22] = 0
    f[:, 22] = 64
    f[:, 23] = t["proto"]
    if ip_csum == "random":
        rng = rng or np.random.default_rng(0)
        f[:, 24:26] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    else:
        f[:, 24:26] = 0
    f[:, 26:30] = t["sip"].astype(">u4").view(np.uint8).reshape(n, 4)
    f[:, 30:34] = t["dip"].astype(">u4").view(np.uint8).reshape(n, 4)
    f[:, 34:36] = t["sport"].astype(">u2").view(np.uint8).reshape(n, 2)
    f[:, 36:38] = t["dport"].astype(">u2").view(np.uint8).reshape(n, 2)
    tcp = t["proto"] == 6
    udp_len = (frame_len - 34).astype(">u2").view(np.uint8).reshape(n, 2)
    u = ~tcp
    f[u, 38:40] = udp_len[u]
    f[tcp, 46] = 0x50  # data offset 5
    f[tcp, 47] = 0x10  # ACK
    f[tcp, 48:50] = np.frombuffer(b"\x20\x00", np.uint8)
    return f


def em_workload(n_rules, n_pkts, hit_frac=0.5, seed=0x5EED, stride=64,
                frame_len=60, out=None, pkt_seed=None):
    """C2/C5-style workload: n_rules distinct 5-tuple rules (gate i % 64),
    n_pkts frames of which hit_frac hit a uniformly chosen rule. The rules
    depend only on `seed`; packets on `pkt_seed` (default: seed)."""
    rng = np.random.default_rng(seed)
    rules = random_tuples(n_rules, rng)
    if pkt_seed is not None:
        rng = np.random.default_rng(pkt_seed)
    keys = tuple_keys(rules)
    gates = (np.arange(n_rules) % 64).astype(np.uint16)
    hit = rng.random(n_pkts) < hit_frac
    idx = rng.integers(0, n_rules, n_pkts)
    pk = random_tuples(n_pkts, rng)
    for fld in pk:
        pk[fld][hit] = rules[fld][idx[hit]]
    frames = build_frames(pk, frame_len, stride, out=out)
    return keys, gates, frames


# --- WildcardMatch (C4) ------------------------------------------------------
# masks over the 5-tuple key (proto|sip|dip|sport|dport), SURVEY §8d
def _m(proto=0, sip=0, dip=0, sport=0, dport=0):
    b = bytearray(16)
    b[0] = proto
    b[1:5] = sip.to_bytes(4, "big")
    b[5:9] = dip.to_bytes(4, "big")
    b[9:11] = sport.to_bytes(2, "big")
    b[11:13] = dport.to_bytes(2, "big")
    return bytes(b)


WM_MASKS = [
    _m(sip=0xFFFFFFFF, dport=0xFFFF),            # /32 src + dport
    _m(dip=0xFFFFFF00),                          # /24 dst
    _m(sip=0xFFFF0000, dip=0xFFFF0000),          # /16 src + /16 dst
    _m(proto=0xFF, dport=0xFFFF),                # proto + dport
    _m(0xFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFF, 0xFFFF),  # full 5-tuple
    _m(sip=0xFFFFFFFF),                          # /32 src
    _m(dip=0xFF000000),                          # /8 dst
    _m(sport=0xFFFF),                            # sport
]


def wm_workload(n_rules, n_pkts, match_frac=0.5, seed=0x5EED, stride=2048,
                sizes=IMIX, prio_range=1000, masks=WM_MASKS):
    """C4-style workload: n_rules (value, mask, priority, gate) over the given
    masks (priorities U[0, prio_range): ties are frequent), IMIX frames of
    which match_frac are derived from rule base tuples."""
    rng = np.random.default_rng(seed)
    base = random_tuples(n_rules, rng)
    bkeys = tuple_keys(base)
    mi = rng.integers(0, len(masks), n_rules)
    marr = np.frombuffer(b"".join(masks), np.uint8).reshape(len(masks), 16)
    rkeys = bkeys & marr[mi]
    prio = rng.integers(0, prio_range, n_rules).astype(np.int32)
    gates = rng.integers(0, 64, n_rules).astype(np.uint16)
    derived = rng.random(n_pkts) < match_frac
    idx = rng.integers(0, n_rules, n_pkts)
    pk = random_tuples(n_pkts, rng)
    for fld in pk:
        pk[fld][derived] = base[fld][idx[derived]]
    lens = np.array([s for s, _ in sizes])
    w = np.array([c for _, c in sizes], np.float64)
    flen = lens[rng.choice(len(lens), n_pkts, p=w / w.sum())]
    frames = build_frames(pk, flen, stride)
    return rkeys, marr[mi], prio, gates, frames, flen


def cksum_workload(n_pkts, frame_len=1496, stride=2048, udp_frac=0.5,
                   seed=0x5EED, payload="random"):
    """C3-style frames: IPv4 + UDP/TCP, random payload, garbage checksums."""
    rng = np.random.default_rng(seed)
    t = random_tuples(n_pkts, rng, protos=(17,))
    t["proto"][rng.random(n_pkts) >= udp_frac] = 6
    f = build_frames(t, frame_len, stride, rng=rng, payload=payload,
                     ip_csum="random")
    # garbage L4 checksum words
    udp = t["proto"] == 17
    f[udp, 40:42] = rng.integers(0, 256, (int(udp.sum()), 2), dtype=np.uint8)
    f[~udp, 50:52] = rng.integers(0, 256, (int((~udp).sum()), 2), dtype=np.uint8)
    return f


def cksum_p11_workload(n, seed=11):
    """Frames whose UDP / TCP length fields run past data_len over non-zero
    bytes: the reference sums udp.length / ip.length-derived
    byte counts from the packet buffer whatever data_len is
    (checksum.h:398-407, 492-504; l4_checksum.cc:61-82). Returns (frames
    n x 2048 -- the whole data area, every byte past the frame random --,
    data_len per packet)."""
    rng = np.random.default_rng(seed)
    f = cksum_workload(n, frame_len=1496, seed=seed)
    f[:, 1496:] = rng.integers(1, 256, (n, 2048 - 1496), dtype=np.uint8)
    lens = rng.integers(60, 1497, n).astype(np.uint16)
    udp = f[:, 23] == 17
    # a third of the frames: length fields out to the end of the data area
    far = rng.random(n) < 1 / 3
    ln = rng.integers(1500, 2048 - 34, n)
    u = far & udp
    f[u, 38] = ln[u] >> 8
    f[u, 39] = ln[u] & 255
    t = far & ~udp
    f[t, 16] = (ln[t] + 20) >> 8
    f[t, 17] = (ln[t] + 20) & 255
    # and some with data_len past what the headers give (nothing to add)
    lens[rng.random(n) < 0.1] = 2048
    return f, lens
