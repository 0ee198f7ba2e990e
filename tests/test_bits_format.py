"""The bitmap hand-back's layout (KWK_COMPACT_BITS, include/kwok_engine.h) on the CPU: the header's
KWK_BITS_SLOT against the 2-byte records' KWK_FIRED16_SLOT of the same id (compiled with gcc), and
abi.bits_decode on lists laid out as bits_kernel writes them (engine.hip).  The device path itself
is checked against kwk_fired in tests/test_scale_properties.py (GPU)."""
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lds_id8(k, lane):
    """lds_id8(k, lane * 4) (engine.hip): the LDS offset of a lane's phase-1 bit k."""
    jj = k & 7
    return jj << 8 | ((lane * 4) ^ (jj << 2)) | (k >> 3)


def test_bits_slot_is_the_record_slot_and_a_bijection():
    from kwok_amd.host import abi
    i = np.arange(2048, dtype=np.uint32)
    x = np.array([_lds_id8(int(v) & 31, int(v) >> 5) for v in i], dtype=np.uint32)
    sl, _, _ = abi.fired16_decode(x.astype(np.uint16), np.array([2048], dtype=np.uint32), 2048)
    assert np.array_equal(sl, abi.bits_slot(i).astype(np.int64))
    assert np.array_equal(np.sort(sl), np.arange(2048))


def test_header_bits_slot_macro(tmp_path):
    src = tmp_path / "m.c"
    src.write_text('#include <stdio.h>\n#include "kwok_engine.h"\n'
                   'int main(void) { for (unsigned i = 0; i < 2048; ++i) printf("%u\\n", KWK_BITS_SLOT(i)); return 0; }\n')
    exe = tmp_path / "m"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = np.array(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split(), dtype=np.int64)
    from kwok_amd.host import abi
    assert np.array_equal(got, abi.bits_slot(np.arange(2048)).astype(np.int64))


def _encode(segs):
    """bits_size_kernel + bits_write_kernel's layout: {c, z} per segment, then per segment the 8
    summary words, the nonzero map bytes (padded to a word) and the stage codes (padded)."""
    head, body = [], []
    for bits, stages in segs:
        m = np.zeros(2048, dtype=np.uint8)
        m[bits] = 1
        mb = np.packbits(m, bitorder="little")  # 256 map bytes
        nz = mb != 0
        head.append(len(bits) | int(nz.sum()) << 16)
        body.append(np.packbits(nz.astype(np.uint8), bitorder="little").view(np.uint32))
        zb = np.zeros(4 * ((int(nz.sum()) + 3) // 4), dtype=np.uint8)
        zb[:int(nz.sum())] = mb[nz]
        body.append(zb.view(np.uint32))
        w = np.zeros((len(bits) + 15) // 16, dtype=np.uint32)
        for j, st in enumerate(stages):
            w[j // 16] |= np.uint32(int(st) << (2 * (j % 16)))
        body.append(w)
    return np.concatenate([np.array(head, dtype=np.uint32)] + body)


def test_bits_decode_round_trip():
    from kwok_amd.host import abi
    rng = np.random.default_rng(7)
    segs = []
    for density in (0.0, 0.1, 0.5, 1.0, 0.01, 0.33):  # empty, ragged and full segments
        bits = np.flatnonzero(rng.random(2048) < density).astype(np.int64)
        segs.append((bits, rng.integers(0, 4, len(bits))))
    words = _encode(segs)
    slot, stage = abi.bits_decode(words, len(segs), 2048)
    want_slot = np.concatenate([s * 2048 + abi.bits_slot(b).astype(np.int64) for s, (b, _) in enumerate(segs)])
    want_stage = np.concatenate([st for _, st in segs]).astype(np.uint32)
    assert np.array_equal(slot, want_slot) and np.array_equal(stage, want_stage)
