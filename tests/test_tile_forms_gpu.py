"""GPU parity of the persistent long-piece kernel forms against the oracle,
bit for bit (NaN payloads included):

* "persist" (psg_tile.hip kP): psg_tile.hip walking an XCD-contiguous run of
  tiles per workgroup, the next tile's push table prefetched into LDS by
  LDS-DMA;
* "staged" (psg_tile_staged.hip, A/B form): each tile's D, bucket index and
  pieces moved into LDS one tile ahead, two workgroups per CU.

Both keep psg_tile.hip's search / order check / wave-ordered fold, so these
cases aim at what the persistent memory side adds: pieces at every 16-B
alignment, D and the job range at odd offsets, partial last tiles, workgroup
runs that cross job boundaries (and push counts), tiles whose pieces exceed
the stage (staged: later push groups staged synchronously), runs with fewer
tiles than workgroups, unsorted pushes, f64 (persist) and the in-kernel
bucket table of context flushes (no resident index).  Reference semantics:
serialSetValue / parallelSetValue (kv_vector.h:84-204) over oldMatch / match
(message.h:134-267).
"""
import numpy as np
import pytest

import oracle_py as O
from test_gpu_parity import ALL, assert_bitexact, plan_for, random_case, run_ctx, to_dev
from test_gpu_parity import torch_cuda  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


FORMS = ["persist", "staged"]


def _flags(form):
    # uniform (push-per-round) rounds forced: jobs of short pieces would take
    # the packed kernel by default
    from parameter_server_amd import _lib
    f = _lib.PSG_FORM_STAGED if form == "staged" else _lib.PSG_FORM_PERSIST | _lib.PSG_NO_STAGED
    return f | _lib.PSG_FORM_UNIFORM


def _kernel(form):
    from parameter_server_amd import _lib
    return _lib.PSG_KERNEL_STAGED if form == "staged" else _lib.PSG_KERNEL_PERSIST


def _check_plan(torch, cases, parallel, form, reps=2, want_form=True, dtype=np.float32):
    plan, keep = plan_for(torch, cases, dtype=dtype, parallel=parallel, flags=_flags(form))
    if want_form:
        assert plan.form == _kernel(form)
    for _ in range(reps):
        plan.run()
        assert plan.matched().tolist() == [k.size for _, ps in cases for k, _ in ps]
        for j, (Dj, pushes) in enumerate(cases):
            _, _, _, want, _ = O.aggregate(Dj, *ALL, pushes, parallel=parallel, dtype=dtype)
            assert_bitexact(keep[4 * j + 3][0].cpu().numpy()[: Dj.size], want[0])
    plan.close()


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("parallel", [False, True])
def test_form_random_jobs(torch_cuda, parallel, form):
    """Random jobs of 1..31 pushes (-0.0, +0.0, denormals, NaN values),
    densities from one key per tile to every key, D sizes with partial last
    tiles, in one batch (workgroup runs cross job boundaries)."""
    cases = []
    for seed, (npush, dens, nD) in enumerate([(1, 0.3, 5000), (8, 0.13, 70000), (31, 0.02, 9000),
                                              (17, 0.5, 4097), (3, 1.0, 2048), (13, 0.001, 30000),
                                              (2, 0.9, 1), (31, 0.25, 3100)]):
        D, pushes = random_case(100 + seed, np.float32, 1, npush, dens, nD)
        pushes = [p for p in pushes if p[0].size]
        if pushes:
            cases.append((D, pushes))
    _check_plan(torch_cuda, cases, parallel, form)


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("parallel", [False, True])
def test_form_cfg2_full_size(torch_cuda, parallel, form):
    """cfg2 at full size, both modes, run twice."""
    from parameter_server_amd import synth
    D, pushes = synth.overlap_pushes(1)
    _check_plan(torch_cuda, [(D, pushes)], parallel, form)


def test_persist_f64_random_jobs(torch_cuda):
    """The persistent form in f64 (the reference apps' double), both modes."""
    cases = []
    for seed, (npush, dens, nD) in enumerate([(8, 0.13, 70000), (31, 0.02, 9000), (32, 0.3, 5000)]):
        D, pushes = random_case(300 + seed, np.float64, 1, npush, dens, nD)
        cases.append((D, [p for p in pushes if p[0].size]))
    for parallel in (False, True):
        _check_plan(torch_cuda, cases, parallel, "persist", dtype=np.float64)


@pytest.mark.parametrize("form", FORMS)
def test_form_overflowing_tiles(torch_cuda, form):
    """Tiles whose pieces exceed the stage (31 pushes holding nearly every
    key of the tile: ~24 K key units) read their pieces from global memory;
    tiles of the same job that fit are staged: bit-exact either way."""
    rng = np.random.default_rng(7)
    D = np.unique(rng.integers(0, 1 << 40, 40000, dtype=np.uint64))
    pushes = []
    for p in range(31):
        sel = rng.random(D.size)
        # dense over the first 10 K slots (overflow), sparse past them (staged)
        keep = np.where(np.arange(D.size) < 10000, sel < 0.97, sel < 0.02)
        k = D[keep]
        v = rng.standard_normal(k.size).astype(np.float32)
        v[::11] = -0.0
        pushes.append((k, [v]))
    for parallel in (False, True):
        _check_plan(torch_cuda, [(D, pushes)], parallel, form, reps=1)


@pytest.mark.parametrize("form", FORMS)
def test_form_unaligned_d_and_values(torch_cuda, form):
    """D, push keys and push values at odd 8-B / 4-B offsets (every 16-B
    phase of a piece's first and last unit), job ranges starting mid-array."""
    torch = torch_cuda
    from parameter_server_amd.kv_vector import MergePlan
    from parameter_server_amd._lib import PSG_F32
    rng = np.random.default_rng(11)
    D = np.unique(rng.integers(0, 1 << 50, 30000, dtype=np.uint64))
    pushes = []
    for p in range(9):
        k = np.sort(rng.choice(D, int(rng.integers(2000, 20000)), replace=False))
        pushes.append((k, [rng.standard_normal(k.size).astype(np.float32)]))
    for doff in (0, 1):
        keep = []
        dD = to_dev(torch, np.concatenate([np.zeros(doff, np.uint64), D]))
        pk, pv = [], []
        for p, (k, vs) in enumerate(pushes):
            ko, vo = (p + doff) % 2, (p + doff) % 4
            tk = to_dev(torch, np.concatenate([np.zeros(ko, np.uint64), k]))
            tv = to_dev(torch, np.concatenate([np.zeros(vo, np.float32), vs[0]]))
            keep += [tk, tv]
            pk.append(tk.data_ptr() + 8 * ko)
            pv.append([tv.data_ptr() + 4 * vo])
        out = torch.full((D.size + 1,), float("nan"), dtype=torch.float32, device="cuda")
        keep += [dD, out]
        job = {"keys": dD.data_ptr() + 8 * doff, "nslots": D.size, "push_keys": pk,
               "push_vals": pv, "push_n": [k.size for k, _ in pushes],
               "out": [out.data_ptr() + 4]}
        for parallel in (False, True):
            plan = MergePlan(0, PSG_F32, 1, [job], parallel, _flags(form))
            assert plan.form == _kernel(form)
            plan.run()
            assert plan.matched().tolist() == [k.size for k, _ in pushes]
            _, _, _, want, _ = O.aggregate(D, *ALL, pushes, parallel=parallel)
            assert_bitexact(out.cpu().numpy()[1: D.size + 1], want[0])
            plan.close()


@pytest.mark.parametrize("form", FORMS)
def test_form_small_and_many_jobs(torch_cuda, form):
    """Fewer tiles than workgroups (one 3-slot job), and 200 jobs of 1-3
    tiles each (every workgroup run crosses jobs of different push counts)."""
    rng = np.random.default_rng(12)
    small = random_case(31, np.float32, 1, 4, 0.7, 3)
    _check_plan(torch_cuda, [(small[0], [p for p in small[1] if p[0].size])], False, form)
    cases = []
    for j in range(200):
        D, pushes = random_case(1000 + j, np.float32, 1, int(rng.integers(1, 32)),
                                float(rng.uniform(0.05, 0.6)), int(rng.integers(1, 3000)))
        pushes = [p for p in pushes if p[0].size]
        if pushes:
            cases.append((D, pushes))
    _check_plan(torch_cuda, cases, True, form, reps=1)


@pytest.mark.parametrize("form", FORMS)
def test_form_unsorted_push_is_reported(torch_cuda, form):
    """An unsorted push (two 300-key blocks swapped) and a push with a key
    outside D are reported unmatched by both forms too."""
    torch = torch_cuda
    from parameter_server_amd import synth
    D, pushes = synth.overlap_pushes(2, npush=4, n=20000)
    k0 = pushes[0][0].copy()
    k0[1000:1300], k0[5000:5300] = pushes[0][0][5000:5300], pushes[0][0][1000:1300]
    k1 = pushes[1][0].copy()
    k1[-1] = D[-1] + np.uint64(1)  # above every server key (still sorted)
    bad = [(k0, pushes[0][1]), (k1, pushes[1][1])] + pushes[2:]
    plan, keep = plan_for(torch, [(D, bad)], flags=_flags(form))
    plan.run()
    mt = plan.matched().tolist()
    assert mt[0] < k0.size and mt[1] < k1.size and mt[2:] == [20000, 20000]
    plan.close()


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("parallel", [False, True])
def test_form_context_flush(torch_cuda, parallel, form):
    """The server API (psg_push / psg_received) with both forms: its
    flushes have no resident bucket index, so the kernel builds each tile's
    table in LDS; a sub-range job, launch seams of 5 pushes (continued
    aggregates run psg_tile.hip) and one launch."""
    D, pushes = random_case(41, np.float32, 1, 12, 0.3, 40000)
    pushes = [p for p in pushes if p[0].size]
    kb, ke = int(D[D.size // 7]), int(D[-(D.size // 9)])
    pushes = [(k[(k >= kb) & (k < ke)], [v[(k >= kb) & (k < ke)] for v in vs]) for k, vs in pushes]
    for flush in (None, 5):
        out = run_ctx(D, pushes, kb, ke, np.float32, parallel, flags=_flags(form), flush=flush)
        _, lo, hi, want, _ = O.aggregate(D, kb, ke, pushes, parallel, 1, np.float32)
        assert tuple(out[0][0]) == (lo, hi)
        assert_bitexact(out[0][1], want[0])
