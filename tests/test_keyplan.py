"""The classify kernels' key build, run on the host through bg_debug_key
(same FieldPlan, same v_perm_b32 byte-permute plan), against the
reference's definition of the key: ExactMatchTable::MakeKeys
(exact_match_table.h:239-263) -- field bytes & mask at key byte `pos`, the
rest zero; WildcardMatch::ProcessBatch (wildcard_match.cc:169-197) -- raw
field bytes. CPU only: validates the plan compiler for random layouts."""
import ctypes as C

import numpy as np
import pytest

from bess_amd import _lib
from bess_amd._lib import bg_field, lib


def expect_key(frame, fields, em_masks):
    key = bytearray(64)
    for off, size, pos, mask in fields:
        v = int.from_bytes(bytes(frame[off:off + size]), "little")
        if em_masks:
            v &= mask
        key[pos:pos + size] = v.to_bytes(size, "little")
    return bytes(key)


def device_key(frame, fields, em_masks):
    arr = (bg_field * len(fields))()
    for i, (off, size, pos, mask) in enumerate(fields):
        arr[i].offset, arr[i].size, arr[i].pos = off, size, pos
        arr[i].attr_id, arr[i].mask = -1, mask
    out = (C.c_uint8 * 64)()
    buf = np.ascontiguousarray(frame)
    rc = lib().bg_debug_key(arr, len(fields), int(em_masks), buf.ctypes.data,
                            out)
    assert rc == 0
    return bytes(out)


def random_layout(rng, spread):
    nf = int(rng.integers(1, 9))
    fields, pos = [], 0
    for _ in range(nf):
        size = int(rng.integers(1, 9))
        off = int(rng.integers(0, spread))
        mask = int(rng.integers(0, 1 << 63)) | int(rng.integers(0, 2)) << 63
        mask &= (1 << (8 * size)) - 1
        fields.append((off, size, pos, mask))
        pos += size
    return fields


@pytest.mark.parametrize("spread", [8, 24, 48, 200, 1024])
def test_key_plan_random_layouts(spread):
    rng = np.random.default_rng(spread)
    for _ in range(300):
        fields = random_layout(rng, spread)
        frame = rng.integers(0, 256, 1024 + 64, dtype=np.uint8)
        for em in (True, False):
            assert device_key(frame, fields, em) == expect_key(frame, fields, em), \
                (fields, em)


def test_key_plan_five_tuple():
    fields = [(23, 1, 0, 0xFF), (26, 4, 1, 0xFFFFFFFF), (30, 4, 5, 0xFFFFFFFF),
              (34, 2, 9, 0xFFFF), (36, 2, 11, 0xFFFF)]
    frame = np.arange(64, dtype=np.uint8)
    assert device_key(frame, fields, True) == expect_key(frame, fields, True)


def test_debug_key_is_declared():
    assert "bg_debug_key" in _lib.declared_symbols()
