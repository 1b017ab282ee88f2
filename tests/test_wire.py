"""Wire ingress: the crc32c key signature of the key cache.

CPU tests pin the oracle's restatement (oracle/psg_oracle.c orc_crc32c_extend)
against the reference's own known answers (src/test/crc32c_test.cc:13-65,
RFC 3720 B.4, held as data in tests/golden/known_answers.json) and against
oracle/_ref/libref_crc32c.so (src/util/crc32c.cc compiled in place).  GPU
tests check psg_crc32c_dev against both, bit-exact.
"""
import json
import os

import numpy as np
import pytest

import oracle_py as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))


def rfc_inputs():
    g = GOLD["crc32c_test"]["standard"]
    pat = {
        "zeros32": bytes(32),
        "ones32": bytes([0xff] * 32),
        "ascending32": bytes(range(32)),
        "descending32": bytes(31 - i for i in range(32)),
    }
    out = []
    for e in g:
        b = pat[e["input"]] if "input" in e else bytes.fromhex(e["input_hex"])
        out.append((b, e["expect"]))
    return out


def test_crc32c_oracle_known_answers():
    for b, want in rfc_inputs():
        assert O.crc32c(b) == want
    g = GOLD["crc32c_test"]
    a, b, whole = (g["extend"][k].encode() for k in ("a", "b", "whole"))
    assert O.crc32c(whole) == O.crc32c(b, O.crc32c(a))
    x, y = (s.encode() for s in g["values_differ"])
    assert O.crc32c(x) != O.crc32c(y)
    c = O.crc32c(g["mask_roundtrip"].encode())
    assert c != O.crc32c_mask(c) and c != O.crc32c_mask(O.crc32c_mask(c))
    assert O.crc32c_unmask(O.crc32c_mask(c)) == c
    assert O.crc32c_unmask(O.crc32c_unmask(O.crc32c_mask(O.crc32c_mask(c)))) == c


@pytest.mark.skipif(not O.ref_crc_available(), reason="oracle/_ref not built (no reference tree)")
def test_crc32c_oracle_vs_reference_build():
    rng = np.random.default_rng(3)
    for n in (0, 1, 3, 4, 5, 15, 16, 17, 31, 64, 1000, 2048, 4099):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        init = int(rng.integers(0, 1 << 32))
        assert O.crc32c(b) == O.ref_crc32c(b)
        assert O.crc32c(b, init) == O.ref_crc32c(b, init)


def test_key_signature_is_prefix_crc():
    keys = np.arange(1000, dtype=np.uint64) * 7919
    assert O.key_signature(keys) == O.crc32c(keys.tobytes()[:2048])
    assert O.key_signature(keys[:10]) == O.crc32c(keys[:10].tobytes())


# ---------------------------------------------------------------- GPU ----
def gpu_crc(torch, segments, max_len=1 << 62, inits=None, align=0):
    """psg_crc32c_dev over byte segments packed into one device buffer (each
    segment starts `align` bytes past a 16-byte boundary)."""
    from parameter_server_amd import _lib
    L = _lib.lib()
    buf = bytearray()
    starts = []
    for s in segments:
        buf += bytes((align - len(buf)) % 16)
        starts.append(len(buf))
        buf += s
    dev = torch.tensor(np.frombuffer(bytes(buf) + bytes(16), np.uint8).copy(), device="cuda")
    out = []
    for i, s in enumerate(segments):
        o = torch.tensor(np.array([starts[i], starts[i] + len(s)], np.uint64).view(np.int64),
                         device="cuda")
        r = torch.zeros(1, dtype=torch.int32, device="cuda")
        ini = None
        if inits is not None:
            ini = torch.tensor(np.array([inits[i]], np.uint32).view(np.int32), device="cuda")
        _lib.check(L.psg_crc32c_dev(dev.data_ptr(), o.data_ptr(), 1, max_len,
                                    None if ini is None else ini.data_ptr(), r.data_ptr(), None))
        out.append(int(r.cpu().numpy().view(np.uint32)[0]))
    return out


@pytest.mark.gpu
def test_gpu_crc32c_known_answers():
    import torch
    assert torch.cuda.is_available()
    cases = rfc_inputs()
    for align in (0, 3, 8):
        got = gpu_crc(torch, [b for b, _ in cases], align=align)
        assert got == [w for _, w in cases]
    g = GOLD["crc32c_test"]
    a, b, whole = (g["extend"][k].encode() for k in ("a", "b", "whole"))
    assert gpu_crc(torch, [b], inits=[O.crc32c(a)]) == [O.crc32c(whole)]


@pytest.mark.gpu
def test_gpu_crc32c_batched_segments_vs_oracle():
    """Many segments of ragged lengths in one launch (the key-signature batch),
    each clamped to max_sig_len; plus lengths around the 16-B block, 1 KB
    round and 64 KB chunk seams, unaligned starts and a multi-chunk segment."""
    import torch
    from parameter_server_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(11)
    lens = [0, 1, 7, 15, 16, 17, 63, 64, 1008, 1023, 1024, 1025, 2047, 2048, 2049, 5000,
            65535, 65536, 65537, 200003]
    lens += list(rng.integers(0, 9000, 300))
    blob = rng.integers(0, 256, int(sum(lens)) + 64, dtype=np.uint8)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + 3  # unaligned starts
    d = torch.tensor(blob, device="cuda")
    doff = torch.tensor(off.view(np.int64), device="cuda")
    inits = rng.integers(0, 1 << 32, len(lens), dtype=np.uint64).astype(np.uint32)
    dinit = torch.tensor(inits.view(np.int32), device="cuda")
    for max_len, use_init in ((1 << 62, False), (2048, False), (1 << 62, True), (70000, True)):
        out = torch.zeros(len(lens), dtype=torch.int32, device="cuda")
        _lib.check(L.psg_crc32c_dev(d.data_ptr(), doff.data_ptr(), len(lens), max_len,
                                    dinit.data_ptr() if use_init else None, out.data_ptr(), None))
        got = out.cpu().numpy().view(np.uint32)
        hb = blob.tobytes()
        for i, n in enumerate(lens):
            s = hb[int(off[i]): int(off[i]) + min(int(n), max_len)]
            want = O.crc32c(s, int(inits[i]) if use_init else 0)
            assert int(got[i]) == want, (i, n, max_len, use_init)


@pytest.mark.gpu
def test_gpu_key_signature_of_pushes():
    """The signature the key cache compares: crc32c over the first 2048 key
    bytes of each push (remote_node.cc:108,163), for the cfg2 push shape."""
    import torch
    from parameter_server_amd import _lib, synth
    L = _lib.lib()
    D, pushes = synth.overlap_pushes(seed=5, npush=8, n=131072)
    keys = np.concatenate([k for k, _ in pushes])
    off = np.concatenate([[0], np.cumsum([8 * k.size for k, _ in pushes])]).astype(np.uint64)
    d = torch.tensor(keys.view(np.int64), device="cuda")
    doff = torch.tensor(off.view(np.int64), device="cuda")
    out = torch.zeros(len(pushes), dtype=torch.int32, device="cuda")
    _lib.check(L.psg_crc32c_dev(d.data_ptr(), doff.data_ptr(), len(pushes), 2048, None,
                                out.data_ptr(), None))
    got = out.cpu().numpy().view(np.uint32)
    assert [int(x) for x in got] == [O.key_signature(k) for k, _ in pushes]
    if O.ref_crc_available():
        assert int(got[0]) == O.ref_crc32c(pushes[0][0].tobytes()[:2048])


# --------------------------------------------------- key cache (GPU) ----
def _kvv(dtype=np.float32):
    from parameter_server_amd.kv_vector import KVVector
    from parameter_server_amd._lib import PSG_F32, PSG_F64
    return KVVector(0, PSG_F32 if dtype == np.float32 else PSG_F64)


def _msg(keys=None, vals=None, t=0, sig=None, has_key=True, erase=False, sender=0,
         rng=(0, (1 << 64) - 1)):
    from parameter_server_amd.kv_vector import Message
    return Message(time=t, key_range=rng, sender=sender,
                   key=np.zeros(0, np.uint64) if keys is None else np.asarray(keys, np.uint64),
                   value=[] if vals is None else [np.asarray(v) for v in vals],
                   key_signature=sig, has_key=has_key, erase_key_cache=erase)


def _bits(a):
    a = np.asarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


@pytest.mark.gpu
def test_key_cache_store_then_restore_bitexact():
    """Iteration 1: each worker's push carries keys + signature (stored in
    that sender's cache); iteration 2: pushes carry only the signature and
    the values, the keys are the resident cached copy.  Both aggregates are
    bit-exact against the oracle and identical to plain pushes."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import synth
    D, pushes = synth.overlap_pushes(seed=21, npush=6, n=20000)
    v = _kvv()
    v.setValue(_msg(D))
    for t in (1, 2):
        for w, (k, vals) in enumerate(pushes):
            sig = O.key_signature(k)
            vv = [x * t for x in vals]
            if t == 1:
                v.setValue(_msg(k, vv, t=t, sig=sig, sender=w))
            else:
                v.setValue(_msg(None, vv, t=t, sig=sig, has_key=False, sender=w))
        (rng, got), = v.received(t)
        rc, lo, hi, want, _ = O.aggregate(D, 0, (1 << 64) - 1, [(k, [x * t for x in vals])
                                                                for k, vals in pushes])
        assert rc == 0 and (lo, hi) == tuple(rng)
        assert np.array_equal(_bits(got), _bits(want[0]))
    assert v.key_cache_bytes() == sum(8 * k.size for k, _ in pushes)
    assert v.key_cache_bytes(2) == 8 * pushes[2][0].size
    v.clear_key_cache(2)
    assert v.key_cache_bytes() == sum(8 * k.size for i, (k, _) in enumerate(pushes) if i != 2)
    v.close()


@pytest.mark.gpu
def test_key_cache_signature_errors_and_erase():
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd._lib import PSGError, PSG_ERR_SIGNATURE, PSG_ERR_NO_TIME
    rng = np.random.default_rng(4)
    D = np.unique(rng.integers(0, 1 << 40, 5000, dtype=np.uint64))
    k = np.sort(rng.choice(D, 700, replace=False))
    x = rng.standard_normal(k.size).astype(np.float32)
    v = _kvv()
    v.setValue(_msg(D))
    sig = O.key_signature(k)
    # carried keys whose crc32c differs from the carried signature: CHECK_EQ
    # (:163), checked on the device (no host wait per message) and reported
    # by received(t); a key-only message is checked before its union
    v.setValue(_msg(k, [x], t=1, sig=sig ^ 1))
    with pytest.raises(PSGError) as e:
        v.received(1)
    assert e.value.status == PSG_ERR_SIGNATURE
    with pytest.raises(PSGError) as e:
        v.setValue(_msg(k, [], t=1, sig=sig ^ 1))
    assert e.value.status == PSG_ERR_SIGNATURE
    v.setValue(_msg(k, [x], t=1, sig=sig))  # a good one at the same time: clean
    (_, got), = v.received(1)
    assert np.array_equal(_bits(got), _bits(O.aggregate(D, 0, (1 << 64) - 1, [(k, [x])])[3][0]))
    v.clear_key_cache()
    # restore without an entry, signature != 0: CHECK_EQ(sig, cache.first) (:174)
    with pytest.raises(PSGError) as e:
        v.setValue(_msg(None, [x], t=1, sig=sig, has_key=False))
    assert e.value.status == PSG_ERR_SIGNATURE
    # restore without an entry, signature 0: no keys -> message ignored (kv_vector.h:177)
    v.setValue(_msg(None, [x], t=1, sig=0, has_key=False))
    with pytest.raises(PSGError) as e:
        v.received(1)
    assert e.value.status == PSG_ERR_NO_TIME
    # store, then a message without signature drops the entry (:143-146)
    v.setValue(_msg(k, [x], t=2, sig=sig))
    assert v.key_cache_bytes() == 8 * k.size
    v.setValue(_msg(k, [x], t=2))  # plain keys, no signature
    v.setValue(_msg(k, [x], t=2, sig=None, erase=True))
    assert v.key_cache_bytes() == 0
    (_, got), = v.received(2)
    rc, _, _, want, _ = O.aggregate(D, 0, (1 << 64) - 1, [(k, [x])] * 3)
    assert np.array_equal(_bits(got), _bits(want[0]))
    # erase_key_cache after a restore (:183)
    v.setValue(_msg(k, [x], t=3, sig=sig))
    v.setValue(_msg(None, [x], t=3, sig=sig, has_key=False, erase=True))
    assert v.key_cache_bytes() == 0
    with pytest.raises(PSGError):
        v.setValue(_msg(None, [x], t=3, sig=sig, has_key=False))
    (_, got), = v.received(3)
    want2 = O.aggregate(D, 0, (1 << 64) - 1, [(k, [x])] * 2)[3][0]
    assert np.array_equal(_bits(got), _bits(want2))
    v.close()


@pytest.mark.gpu
def test_key_cache_bad_signature_is_never_restored():
    """The reference checks a carried signature before it stores the keys
    (remote_node.cc:161-165).  Here a keys + values message is checked on the
    device after return; the entry it stored is pending on that check, so a
    later signature-only message with the same signature must fail (and the
    entry is dropped) instead of restoring keys that never matched.  The same
    holds when the keyed message itself failed a later host check (values
    size), and a good entry restores after its check passed."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd._lib import PSGError, PSG_ERR_SIGNATURE, PSG_ERR_SIZE
    rng = np.random.default_rng(14)
    D = np.unique(rng.integers(0, 1 << 40, 6000, dtype=np.uint64))
    k = np.sort(rng.choice(D, 800, replace=False))
    x = rng.standard_normal(k.size).astype(np.float32)
    v = _kvv()
    v.setValue(_msg(D))
    bad = O.key_signature(k) ^ 0x5A5A
    v.setValue(_msg(k, [x], t=1, sig=bad, sender=3))  # stored pending, check fails on the device
    with pytest.raises(PSGError) as e:
        v.setValue(_msg(None, [x], t=2, sig=bad, has_key=False, sender=3))
    assert e.value.status == PSG_ERR_SIGNATURE
    assert v.key_cache_bytes(3) == 0  # the entry was dropped
    with pytest.raises(PSGError) as e:
        v.received(1)
    assert e.value.status == PSG_ERR_SIGNATURE
    # a keyed message that fails its values-size check after storing
    with pytest.raises(PSGError) as e:
        v.setValue(_msg(k, [x[:-1]], t=3, sig=bad, sender=4))
    assert e.value.status == PSG_ERR_SIZE
    with pytest.raises(PSGError) as e:
        v.setValue(_msg(None, [x], t=3, sig=bad, has_key=False, sender=4))
    assert e.value.status == PSG_ERR_SIGNATURE
    # stored and erased by the same message (:183): the one device check is
    # still counted into the aggregate and reported by received(t)
    v.setValue(_msg(k, [x], t=4, sig=bad, sender=6, erase=True))
    assert v.key_cache_bytes(6) == 0
    with pytest.raises(PSGError) as e:
        v.received(4)
    assert e.value.status == PSG_ERR_SIGNATURE
    # a good signature: stored pending, restored once its check passed
    good = O.key_signature(k)
    v.setValue(_msg(k, [x], t=5, sig=good, sender=5))
    v.setValue(_msg(None, [x], t=5, sig=good, has_key=False, sender=5))
    (_, got), = v.received(5)
    want = O.aggregate(D, 0, (1 << 64) - 1, [(k, [x])] * 2)[3][0]
    assert np.array_equal(_bits(got), _bits(want))
    v.close()


@pytest.mark.gpu
def test_key_cache_many_pending_checks_share_counter_slabs():
    """More stored-pending entries than one counter slab holds (256): each
    keeps its own pooled counter; one bad entry among them is caught at its
    restore and the rest restore bit-exactly."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd._lib import PSGError, PSG_ERR_SIGNATURE
    rng = np.random.default_rng(21)
    D = np.unique(rng.integers(0, 1 << 40, 4000, dtype=np.uint64))
    v = _kvv()
    v.setValue(_msg(D))
    nsend, badsend = 300, 277
    ks = [np.sort(rng.choice(D, 64, replace=False)) for _ in range(nsend)]
    xs = [rng.standard_normal(64).astype(np.float32) for _ in range(nsend)]
    for s in range(nsend):
        sig = O.key_signature(ks[s]) ^ (1 if s == badsend else 0)
        v.setValue(_msg(ks[s], [xs[s]], t=1, sig=sig, sender=s))
    with pytest.raises(PSGError):
        v.received(1)  # the bad one counted into the aggregate
    for s in range(nsend):
        sig = O.key_signature(ks[s]) ^ (1 if s == badsend else 0)
        if s == badsend:
            with pytest.raises(PSGError) as e:
                v.setValue(_msg(None, [xs[s]], t=2, sig=sig, has_key=False, sender=s))
            assert e.value.status == PSG_ERR_SIGNATURE
        else:
            v.setValue(_msg(None, [xs[s]], t=2, sig=sig, has_key=False, sender=s))
    (_, got), = v.received(2)
    want = O.aggregate(D, 0, (1 << 64) - 1,
                       [(ks[s], [xs[s]]) for s in range(nsend) if s != badsend])[3][0]
    assert np.array_equal(_bits(got), _bits(want))
    v.close()


@pytest.mark.gpu
def test_key_cache_replaced_while_pushes_pending_and_key_only():
    """An entry replaced (new keys, same channel/range) while pushes restored
    from the old one are still pending: those pushes keep the old resident
    keys.  A key-only message restored from the cache is a setUnion."""
    import torch
    assert torch.cuda.is_available()
    rng = np.random.default_rng(8)
    D = np.unique(rng.integers(0, 1 << 40, 8000, dtype=np.uint64))
    k1 = np.sort(rng.choice(D, 900, replace=False))
    k2 = np.sort(rng.choice(D, 1300, replace=False))
    x1 = rng.standard_normal(k1.size).astype(np.float64)
    x2 = rng.standard_normal(k2.size).astype(np.float64)
    v = _kvv(np.float64)
    v.setValue(_msg(D))
    v.setValue(_msg(k1, [x1], t=5, sig=O.key_signature(k1)))
    v.setValue(_msg(None, [x1], t=5, sig=O.key_signature(k1), has_key=False))
    v.setValue(_msg(k2, [x2], t=5, sig=O.key_signature(k2)))  # replaces the entry
    v.setValue(_msg(None, [x2], t=5, sig=O.key_signature(k2), has_key=False))
    (_, got), = v.received(5)
    _, _, _, want, _ = O.aggregate(D, 0, (1 << 64) - 1, [(k1, [x1]), (k1, [x1]), (k2, [x2]),
                                                         (k2, [x2])], dtype=np.float64)
    assert np.array_equal(_bits(got), _bits(want[0]))
    extra = np.sort(rng.integers(1 << 41, 1 << 42, 50, dtype=np.uint64))
    v.setValue(_msg(extra, None, sig=O.key_signature(extra), sender=3))
    assert np.array_equal(v.key(0), O.set_union(D, extra))
    v.setValue(_msg(None, None, sig=O.key_signature(extra), has_key=False, sender=3))
    assert np.array_equal(v.key(0), O.set_union(D, extra))
    v.close()


@pytest.mark.gpu
def test_pinned_and_pageable_pushes_agree():
    """Pushes from pinned host memory (direct DMA) and from pageable memory
    (staging ring) give the same bits; the caller may overwrite its buffers
    right after psg_push returns."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import synth
    D, pushes = synth.overlap_pushes(seed=13, npush=8, n=131072)
    outs = []
    for pinned in (False, True):
        v = _kvv()
        v.setValue(_msg(D))
        kbuf = torch.empty(131072, dtype=torch.int64, pin_memory=pinned).numpy().view(np.uint64)
        vbuf = torch.empty(131072, dtype=torch.float32, pin_memory=pinned).numpy()
        for k, vals in pushes:
            kb, vb = kbuf[: k.size], vbuf[: k.size]
            kb[:] = k
            vb[:] = vals[0]
            v.setValue(_msg(kb, [vb], t=9))
            kb[:] = 0  # reuse the buffers at once
            vb[:] = np.nan
        (_, got), = v.received(9)
        outs.append(got)
        v.close()
    _, _, _, want, _ = O.aggregate(D, 0, (1 << 64) - 1, pushes)
    for got in outs:
        assert np.array_equal(_bits(got), _bits(want[0]))


@pytest.mark.gpu
def test_pinned_offsets_zero_copy():
    """Pinned pushes are read by the GPU itself (zero-copy kernel) when both
    ends are 16-B aligned, by a DMA copy otherwise: buffers that start inside
    a pinned allocation (aligned and unaligned offsets, odd lengths) give the
    oracle's bits."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import synth
    D, pushes = synth.overlap_pushes(seed=19, npush=6, n=30001)
    tot = sum(k.size for k, _ in pushes) + 64 * len(pushes)
    from parameter_server_amd import _lib
    _, _, _, want, _ = O.aggregate(D, 0, (1 << 64) - 1, pushes)
    for hold in (False, True):  # hold: the aligned ones go in one batched launch
        kall = torch.zeros(tot, dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
        vall = torch.zeros(tot, dtype=torch.float32, pin_memory=True).numpy()
        v = _kvv()
        if hold:
            _lib.check(v._L.psg_set_match_flags(v._h, _lib.PSG_SERIAL_MATCH |
                                                _lib.PSG_HOLD_BUFFERS))
        v.setValue(_msg(D))
        at = 0
        for p, (k, vals) in enumerate(pushes):
            ko = at + (2 if p % 2 == 0 else 1)  # 16-B aligned / 8-B aligned keys
            vo = at + (4 if p % 3 else 1)       # 16-B aligned / 4-B aligned values
            kb, vb = kall[ko: ko + k.size], vall[vo: vo + k.size]
            kb[:] = k
            vb[:] = vals[0]
            v.setValue(_msg(kb, [vb], t=3))
            at += k.size + 64
        (_, got), = v.received(3)
        v.close()
        assert np.array_equal(_bits(got), _bits(want[0])), hold


@pytest.mark.gpu
def test_received_into_pinned_output():
    """received(t) into pinned host arrays: when one launch covers the
    aggregate the merge kernel writes the sums there itself; at an unaligned
    start it falls back to a readback.  f64 with m = 2 and f32 with m = 1."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import synth
    from parameter_server_amd.kv_vector import KVVector, Message
    from parameter_server_amd._lib import PSG_F32, PSG_F64
    D, pushes = synth.overlap_pushes(seed=23, npush=4, n=20000)
    rng = np.random.default_rng(23)
    for dt, code, m in ((np.float64, PSG_F64, 2), (np.float32, PSG_F32, 1)):
        vals = [[rng.standard_normal(k.size).astype(dt) for _ in range(m)] for k, _ in pushes]
        _, _, _, want, _ = O.aggregate(D, 0, (1 << 64) - 1,
                                       [(k, v) for (k, _), v in zip(pushes, vals)], False, 1, dt)
        tdt = torch.float64 if dt == np.float64 else torch.float32
        for off in (0, 1):  # 16-B aligned start / unaligned start (readback)
            v = KVVector(0, code)
            v.setValue(Message(key=D))
            for (k, _), x in zip(pushes, vals):
                v.setValue(Message(time=5, key=k, value=x))
            buf = [torch.full((D.size + 2,), np.nan, dtype=tdt, pin_memory=True).numpy()
                   for _ in range(m)]
            out = v.received(5, out=[b[off:] for b in buf])
            v.close()
            for i in range(m):
                assert out[i][1].ctypes.data == buf[i][off:].ctypes.data  # written in place
                assert np.array_equal(_bits(out[i][1]), _bits(want[i])), (dt, off, i)


@pytest.mark.gpu
def test_hold_buffers_option():
    """PSG_HOLD_BUFFERS: pinned push buffers are DMA'd without a wait per
    push and must stay valid until received(t); the result is unchanged."""
    import ctypes as C
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import synth, _lib
    from parameter_server_amd.kv_vector import KVVector
    D, pushes = synth.overlap_pushes(seed=17, npush=8, n=60000)
    v = KVVector(0)
    _lib.check(v._L.psg_set_match_flags(v._h, _lib.PSG_SERIAL_MATCH | _lib.PSG_HOLD_BUFFERS))
    v.setValue(_msg(D))
    held = [(torch.from_numpy(k.view(np.int64)).pin_memory().numpy().view(np.uint64),
             torch.from_numpy(x[0]).pin_memory().numpy()) for k, x in pushes]
    for t in (1, 2):
        for k, x in held:
            v.setValue(_msg(k, [x * 1.0 if t == 2 else x], t=t))
        (_, got), = v.received(t)
        _, _, _, want, _ = O.aggregate(D, 0, (1 << 64) - 1, pushes)
        assert np.array_equal(_bits(got), _bits(want[0]))
    v.close()


# ------------------------------------------------------------- snappy ----
# Spec-derived known answers (snappy format_description.txt; no snappy
# vectors ship with the reference): preamble varint, literal, copy-1,
# overlapping copy-2 (run length), a 4-byte-offset copy, long literals.
SNAPPY_KNOWN = [
    (bytes([0x0b, 0x28]) + b"hello world", b"hello world"),
    # "abc" literal + copy of 9 at offset 3 (1-byte offset tag 0x15)
    (bytes([0x0c, 0x08]) + b"abc" + bytes([0x15, 0x03]), b"abcabcabcabc"),
    # "a" + copy-2 of 20 at offset 1 (run of 'a'), tag 2 | (19 << 2)
    (bytes([0x15, 0x00]) + b"a" + bytes([2 | (19 << 2), 0x01, 0x00]), b"a" * 21),
    # "xy" + copy-4 of 6 at offset 2, tag 3 | (5 << 2)
    (bytes([0x08, 0x04]) + b"xy" + bytes([3 | (5 << 2), 2, 0, 0, 0]), b"xyxyxyxy"),
    # a 61..256-byte literal: tag 60 << 2, one length byte (len - 1)
    (bytes([0xc8, 0x01, 60 << 2, 199]) + bytes(range(200)), bytes(range(200))),
]


def test_snappy_oracle_known_and_roundtrip():
    for comp, want in SNAPPY_KNOWN:
        assert O.snappy_uncompress(comp) == want
    rng = np.random.default_rng(2)
    keys = np.sort(rng.integers(0, 1 << 40, 20000, dtype=np.uint64)).tobytes()
    nanrun = np.full(5000, np.nan).view(np.uint64)
    nanrun[:] = np.uint64(0xFFFFFFFFFFFFFFFF)  # Darling's inactive sentinel compresses
    for data in (b"", b"a", keys, nanrun.tobytes(), rng.integers(0, 256, 200000, dtype=np.uint8).tobytes(),
                 b"abcd" * 70000):
        c = O.snappy_compress(data)
        assert O.snappy_uncompress(c) == data
    assert len(O.snappy_compress(nanrun.tobytes())) < 4000
    # corrupt: offset beyond the output, truncated literal, length mismatch
    assert O.snappy_uncompress(bytes([0x04, 0x01, 0x05])) is None
    assert O.snappy_uncompress(bytes([0x05, 0x10, 0x61])) is None
    assert O.snappy_uncompress(bytes([0x06, 0x04]) + b"ab") is None


def _gpu_snappy(parts, caps):
    import torch
    from parameter_server_amd import _lib
    L = _lib.lib()
    soff = np.concatenate([[0], np.cumsum([len(p) for p in parts])]).astype(np.uint64)
    doff = np.concatenate([[0], np.cumsum(caps)]).astype(np.uint64)
    blob = b"".join(parts) + b"\0"
    ds = torch.tensor(np.frombuffer(blob, np.uint8).copy(), device="cuda")
    dd = torch.zeros(int(doff[-1]) + 1, dtype=torch.uint8, device="cuda")
    dso = torch.tensor(soff.view(np.int64), device="cuda")
    ddo = torch.tensor(doff.view(np.int64), device="cuda")
    st = torch.full((len(parts),), 7, dtype=torch.int32, device="cuda")
    _lib.check(L.psg_snappy_uncompress_dev(ds.data_ptr(), dso.data_ptr(), len(parts),
                                           dd.data_ptr(), ddo.data_ptr(), st.data_ptr(), None))
    out = dd.cpu().numpy().tobytes()
    return [out[int(doff[i]):int(doff[i + 1])] for i in range(len(parts))], st.cpu().tolist()


@pytest.mark.gpu
def test_gpu_snappy_batched_parts_vs_oracle():
    """Many message parts in one launch: the spec-derived streams, the
    oracle compressor's output for key arrays, f32/f64 values, NaN-sentinel
    runs, random bytes (literals of every length encoding), multi-block
    (> 64 KB) parts and an empty part -- byte-exact; corrupt parts report
    PSG_ERR_ARG / PSG_ERR_SIZE without disturbing their neighbours."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(4)
    datas = [w for _, w in SNAPPY_KNOWN]
    parts = [c for c, _ in SNAPPY_KNOWN]
    extra = [np.sort(rng.integers(0, 1 << 40, 30000, dtype=np.uint64)).tobytes(),
             rng.standard_normal(40000).astype(np.float32).tobytes(),
             np.full(70000, 0xFFFFFFFFFFFFFFFF, np.uint64).tobytes(),
             rng.integers(0, 256, 300000, dtype=np.uint8).tobytes(),
             (b"parameter server " * 20000),
             b""]
    for d in extra:
        datas.append(d)
        parts.append(O.snappy_compress(d))
    # hand-built: a 70,000-byte literal (3-byte length), then 4-byte-offset
    # copies reaching past the 64 KB ring (69,000 back) and inside it, and a
    # run-length copy (offset 1): the decoder's far path reads its own
    # earlier output from global memory
    lit = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    want = bytearray(lit)
    for off, ln in ((69000, 64), (65537, 33), (100, 64), (1, 40)):
        for _ in range(ln):
            want.append(want[len(want) - off])
    ulen, pre = len(want), bytearray()
    while True:
        pre.append((ulen & 0x7F) | (0x80 if ulen > 0x7F else 0))
        ulen >>= 7
        if not ulen:
            break
    s = pre + bytes([62 << 2]) + (len(lit) - 1).to_bytes(3, "little") + lit
    for off, ln in ((69000, 64), (65537, 33), (100, 64), (1, 40)):
        s += bytes([(ln - 1) << 2 | 3]) + off.to_bytes(4, "little")
    assert O.snappy_uncompress(bytes(s)) == bytes(want)
    datas.append(bytes(want))
    parts.append(bytes(s))
    got, st = _gpu_snappy(parts, [len(d) for d in datas])
    assert st == [0] * len(parts)
    for g, d in zip(got, datas):
        assert g == d
    # the same parts six times over: a launch of more than 64 parts skips the
    # L2 prefetch of each part (psg_snappy.hip kPrefetchParts)
    many = parts * 6
    assert len(many) > 64
    got, st = _gpu_snappy(many, [len(d) for d in datas] * 6)
    assert st == [0] * len(many)
    for g, d in zip(got, datas * 6):
        assert g == d
    # corrupt parts among good ones
    bad = [bytes([0x04, 0x01, 0x05]), parts[1], bytes([0x06, 0x04]) + b"ab", parts[0]]
    got, st = _gpu_snappy(bad, [4, 12, 6, 11])
    assert st[0] == _lib.PSG_ERR_ARG and st[2] == _lib.PSG_ERR_ARG
    assert st[1] == 0 and got[1] == datas[1] and st[3] == 0 and got[3] == datas[0]
    got, st = _gpu_snappy([parts[0]], [12])  # declared 11 bytes, caller expects 12
    assert st == [_lib.PSG_ERR_SIZE]


def _snappy_stream(elems):
    """A raw snappy stream from ("lit", bytes) / ("copy", offset, length)
    elements (length <= 64; 2-byte offsets below 65536, else 4-byte), and
    the bytes it decodes to."""
    out = bytearray()
    body = bytearray()
    for e in elems:
        if e[0] == "lit":
            d = e[1]
            x = len(d) - 1
            if x < 60:
                body.append(x << 2)
            else:
                nb = 1 if x < 256 else 2 if x < 65536 else 3
                body.append((59 + nb) << 2)
                body += x.to_bytes(nb, "little")
            body += d
            out += d
        else:
            _, off, ln = e
            if off < 65536:
                body += bytes([(ln - 1) << 2 | 2]) + off.to_bytes(2, "little")
            else:
                body += bytes([(ln - 1) << 2 | 3]) + off.to_bytes(4, "little")
            for _ in range(ln):
                out.append(out[len(out) - off])
    ulen, pre = len(out), bytearray()
    while True:
        pre.append((ulen & 0x7F) | (0x80 if ulen > 0x7F else 0))
        ulen >>= 7
        if not ulen:
            break
    return bytes(pre + body), bytes(out)


@pytest.mark.gpu
def test_gpu_snappy_deferred_literals():
    """The parse defers literals of >= 2048 bytes to the chip-wide copy
    kernel: copies that read back into them (wholly, straddling a deferred
    literal and ring bytes, run-length, past the 64 KB ring), more deferred
    literals than a part keeps (> 64: the rest move in the parse), literals
    just under the threshold, and destinations at every alignment."""
    rng = np.random.default_rng(8)
    parts, datas = [], []
    for variant in range(4):
        el = []
        nlit = 80 if variant == 0 else 12
        for i in range(nlit):
            ln = int(rng.choice([2047, 2048, 2049, 3000, 4096 + 13, 65536]))
            el.append(("lit", rng.integers(0, 256, ln, dtype=np.uint8).tobytes()))
            if i:
                # back into the previous literal, straddling into this one,
                # run-length, short literal between
                el.append(("copy", ln + 5, 64))
                el.append(("copy", 40, 64))
                el.append(("copy", 1, 17))
                el.append(("lit", rng.integers(0, 256, 9, dtype=np.uint8).tobytes()))
                el.append(("copy", 3000, 33))
        if variant == 1:
            el.append(("copy", 70000, 64))  # past the ring, into a deferred literal
        comp, want = _snappy_stream(el)
        assert O.snappy_uncompress(comp) == want
        parts.append(comp)
        datas.append(want)
    # an odd-sized lead part shifts every later destination's alignment
    lead = _snappy_stream([("lit", b"xyz")])
    parts.insert(0, lead[0])
    datas.insert(0, lead[1])
    got, st = _gpu_snappy(parts, [len(d) for d in datas])
    assert st == [0] * len(parts)
    for g, d in zip(got, datas):
        assert g == d
    # the large cfg2-shaped part: incompressible keys, one literal per block
    big = np.sort(rng.integers(0, 1 << 63, 131072, dtype=np.uint64)).tobytes()
    got, st = _gpu_snappy([O.snappy_compress(big)] * 3, [len(big)] * 3)
    assert st == [0, 0, 0] and all(g == big for g in got)


@pytest.mark.gpu
def test_gpu_snappy_offsets_past_the_ring_and_many_deferred():
    """The 8 KB output ring: element-dense parts (16-byte literals and copies
    of every length 1..64) whose copies reach inside the ring, just past it
    (8,193 .. 65,535 back: 2-byte offsets, read from global memory after a
    flush) and far past it (4-byte offsets); many such parts at once (the
    launch keeps ten parts per CU); and a part with more deferred literals
    (>= 2048 bytes) than its 256-piece list holds, so the rest move in the
    parse -- byte-exact against the spec oracle."""
    rng = np.random.default_rng(12)
    parts, datas = [], []
    for v in range(24):
        el, o = [], 0
        while o < 200_000:
            el.append(("lit", rng.integers(0, 256, 16, dtype=np.uint8).tobytes()))
            o += 16
            band = int(rng.integers(0, 4))
            hi = [64, 8192, 65535, 200_000][band]
            lo = [1, 65, 8193, 65536][band]
            if o > lo:
                off = int(rng.integers(lo, min(hi, o) + 1))
                ln = int(rng.integers(1, 65))
                el.append(("copy", off, ln))
                o += ln
        comp, want = _snappy_stream(el)
        parts.append(comp)
        datas.append(want)
    el = [("lit", rng.integers(0, 256, 12000, dtype=np.uint8).tobytes())]
    for i in range(300):
        el.append(("lit", rng.integers(0, 256, int(rng.choice([2048, 2100, 4096])),
                                       dtype=np.uint8).tobytes()))
        el.append(("copy", 2500, 64))
        el.append(("copy", 9000, 17))
    comp, want = _snappy_stream(el)
    assert O.snappy_uncompress(comp) == want
    parts.append(comp)
    datas.append(want)
    assert O.snappy_uncompress(parts[0]) == datas[0]
    got, st = _gpu_snappy(parts, [len(d) for d in datas])
    assert st == [0] * len(parts)
    for g, d in zip(got, datas):
        assert g == d


@pytest.mark.gpu
def test_gpu_push_compressed_matches_plain_push():
    """psg_push_compressed: snappy parts off the wire (keys + m value parts),
    decompressed on the device and merged -- the same bits as plain pushes;
    a corrupt part (reported by received) and inconsistent part sizes (at
    the push) are refused."""
    import ctypes as C
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib, synth
    from parameter_server_amd.kv_vector import KVVector, Message
    D, pushes = synth.overlap_pushes(seed=33, npush=6, n=50000)
    v = KVVector(0)
    v.setValue(Message(key=D))
    L = v._L

    def cpush(t, k, vals, corrupt=False):
        ck = O.snappy_compress(np.ascontiguousarray(k).tobytes())
        if corrupt:
            ck = ck[:len(ck) // 2]
        cv = [O.snappy_compress(np.ascontiguousarray(x).tobytes()) for x in vals]
        bufs = [C.create_string_buffer(b, len(b)) for b in cv]
        arr = _lib.ptr_array([C.cast(b, C.c_void_p).value for b in bufs])
        sizes = (C.c_size_t * len(cv))(*[len(b) for b in cv])
        return L.psg_push_compressed(v._h, 0, t, 0, (1 << 64) - 1, ck, len(ck), len(cv), arr,
                                     sizes)

    for k, vals in pushes:
        _lib.check(cpush(3, k, vals))
    (_, got), = v.received(3)
    _, _, _, want, _ = O.aggregate(D, 0, (1 << 64) - 1, pushes)
    assert np.array_equal(got.view(np.uint32), want[0].view(np.uint32))
    k, vals = pushes[0]
    # a corrupt part decodes asynchronously: psg_received of its time
    # reports it (PSG_ERR_ARG), beside good pushes of the same time
    _lib.check(cpush(4, pushes[1][0], pushes[1][1]))
    assert cpush(4, k, vals, corrupt=True) == _lib.PSG_OK
    with pytest.raises(_lib.PSGError) as e:
        v.received(4)
    assert e.value.status == _lib.PSG_ERR_ARG
    # declared sizes are checked on the host, at the push
    assert cpush(5, k, [vals[0][:-1]]) == _lib.PSG_ERR_SIZE
    # the context goes on: a later time merges as before
    for kk, vv in pushes[:2]:
        _lib.check(cpush(6, kk, vv))
    (_, got), = v.received(6)
    _, _, _, want, _ = O.aggregate(D, 0, (1 << 64) - 1, pushes[:2])
    assert np.array_equal(got.view(np.uint32), want[0].view(np.uint32))
    v.close()


@pytest.mark.gpu
def test_gpu_snappy_streamed_and_per_wave_forms_agree():
    """Launches of <= 64 parts take the streamed decoder (the compressed
    bytes stream through a 128 KB LDS ring; the parse's own output is staged
    in LDS), larger launches the per-wave one: the same streams decoded both
    ways, byte-exact against the spec oracle.  The streams mix long literals
    (>= 16 KB: the stream restarts past each) with short literals and copies
    that reach back across the restarts (into skipped input: read from
    memory), into staged and into already written-out output, run-length
    copies, 4-byte offsets, and parts starting at every 16-B phase."""
    rng = np.random.default_rng(31)
    parts, datas = [], []
    for v in range(6):
        el, o = [], 0
        while o < 400_000:
            kind = int(rng.integers(0, 6))
            if kind == 0:
                ln = int(rng.choice([16384, 20000, 65536, 70001]))
            elif kind == 1:
                ln = int(rng.integers(600, 4000))
            else:
                ln = int(rng.integers(1, 61))
            el.append(("lit", rng.integers(0, 256, ln, dtype=np.uint8).tobytes()))
            o += ln
            for _ in range(int(rng.integers(0, 3))):
                off = int(rng.integers(1, min(o, 150_000) + 1))
                cl = int(rng.integers(1, 65))
                el.append(("copy", off, cl))
                o += cl
        comp, want = _snappy_stream(el)
        assert O.snappy_uncompress(comp) == want
        parts.append(comp)
        datas.append(want)
    # odd-sized leading parts shift the later parts' 16-B phase
    leads = [_snappy_stream([("lit", bytes(range(i + 1)))]) for i in range(5)]
    streamed = [c for c, _ in leads] + parts
    want_all = [d for _, d in leads] + datas
    got, st = _gpu_snappy(streamed, [len(d) for d in want_all])
    assert st == [0] * len(streamed)
    assert all(g == d for g, d in zip(got, want_all))
    # the same parts in a launch of 70 (> 64: the per-wave decoder)
    filler = [_snappy_stream([("lit", bytes([i]) * 3)]) for i in range(70 - len(streamed))]
    many = streamed + [c for c, _ in filler]
    want_many = want_all + [d for _, d in filler]
    got, st = _gpu_snappy(many, [len(d) for d in want_many])
    assert st == [0] * len(many)
    assert all(g == d for g, d in zip(got, want_many))


@pytest.mark.gpu
def test_gpu_snappy_table_form_paths():
    """Launches of <= 64 parts take the table form (psg_snappy.hip
    snappy_tab_kernel): the tags walked into an LDS table, then every copy
    byte resolved on its own lane through the table to the literal byte it
    repeats.  Parts that exercise each of its paths, byte-exact against the
    spec oracle: copies of copies (chains of depth 1..7: the deeper ones
    written in order by the last step), copies straddling two literals and
    overlapping their own output, copies into deferred (>= 512 B) literals,
    a run of more than 64 unresolved copies (the whole part falls back to the
    streamed form), a part of more than 4,096 elements (falls back before any
    byte moves), and corrupt parts beside good ones."""
    from parameter_server_amd import _lib
    rng = np.random.default_rng(77)
    lit = lambda n: ("lit", rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    parts, datas = [], []
    # chains: each copy repeats the previous one (depth grows by one each)
    el = [lit(1000), ("copy", 1000, 64)]
    for _ in range(6):
        el.append(("copy", 64, 64))
    el += [lit(30), ("copy", 500, 40)]
    parts.append(el)
    # straddling and overlapping copies, deferred literals read back
    el = [lit(100), lit(100), ("copy", 150, 64), ("copy", 30, 64), lit(700), ("copy", 650, 64),
          ("copy", 1, 64), lit(5000), ("copy", 4000, 64), ("copy", 5100, 50), ("copy", 7, 9)]
    parts.append(el)
    # a run: "a" then 100 copies of offset 1 (chains too deep: > 64 unresolved)
    parts.append([("lit", b"a")] + [("copy", 1, 64)] * 100)
    # element-dense: 5,000 three-byte literals and short copies
    el = []
    for i in range(5000):
        el.append(lit(3))
        if i > 10 and i % 3 == 0:
            el.append(("copy", int(rng.integers(1, 30)), int(rng.integers(1, 20))))
    parts.append(el)
    # incompressible-shaped: long literals and spurious 4-byte matches
    el = []
    o = 0
    for _ in range(60):
        n = int(rng.integers(1500, 4000))
        el.append(lit(n))
        o += n
        el.append(("copy", int(rng.integers(4, min(o, 65535))), 4))
        o += 4
    parts.append(el)
    streams = [_snappy_stream(e) for e in parts]
    for c, d in streams:
        assert O.snappy_uncompress(c) == d
    comps = [c for c, _ in streams]
    datas = [d for _, d in streams]
    got, st = _gpu_snappy(comps, [len(d) for d in datas])
    assert st == [0] * len(comps)
    for g, d in zip(got, datas):
        assert g == d
    # corrupt parts between good ones: the table walk reports them
    bad = [comps[0], bytes([0x04, 0x01, 0x05]), comps[1], bytes([0x06, 0x04]) + b"ab", comps[4]]
    got, st = _gpu_snappy(bad, [len(datas[0]), 4, len(datas[1]), 6, len(datas[4])])
    assert st[1] == _lib.PSG_ERR_ARG and st[3] == _lib.PSG_ERR_ARG
    assert st[0] == st[2] == st[4] == 0
    assert got[0] == datas[0] and got[2] == datas[1] and got[4] == datas[4]
    got, st = _gpu_snappy([comps[0]], [len(datas[0]) + 1])
    assert st == [_lib.PSG_ERR_SIZE]
