"""The library's stable (uint64 key, int32 value) pair sort against numpy's
stable argsort, on every path the dispatcher takes (sort.hip
radix_sort_pairs_batched): the one-workgroup LDS sort (seglen <= 4,096), the
sample sort (2^16 <= seglen <= 2^19, more than four 8-bit digits), its
per-bucket radix fallback (a bucket the sample missed), and the one-sweep
radix sort (4,096 < seglen < 2^16, larger, or fewer digits).

The sort carries every ordering the NSGA-II path makes -- objective ranks,
the lexicographic order of the fitnesses, crowding and the last-front cut
(deap/tools/emo.py:38-48, 121-143 use Python's stable ``sorted``) -- so it
has to be exactly the stable order: ties by input position."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LS_CAP = 4096
SS_SAMPLE = 4096


def _sort(gpu, keys, vals, nseg, seglen, begin=0, end=64):
    import torch
    from deap_amd import _lib
    from deap_amd.device import Context
    lib = _lib.load()
    fn = lib.dm_test_sort_pairs
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                   ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    k = torch.from_numpy(keys.view(np.int64).copy()).to(gpu)
    v = torch.from_numpy(vals.copy()).to(gpu)
    ctx = Context.get(gpu)
    _lib.check(fn(ctx.handle, ctypes.c_void_p(k.data_ptr()), ctypes.c_void_p(v.data_ptr()),
                  nseg, seglen, begin, end), "dm_test_sort_pairs")
    return k.cpu().numpy().view(np.uint64), v.cpu().numpy()


def _expect(keys, vals, nseg, seglen, begin, end):
    width = end - begin
    mask = np.uint64(0xFFFFFFFFFFFFFFFF) if width >= 64 else np.uint64((1 << width) - 1)
    ek, ev = keys.copy(), vals.copy()
    for g in range(nseg):
        sl = slice(g * seglen, (g + 1) * seglen)
        bits = (keys[sl] >> np.uint64(begin)) & mask
        o = np.argsort(bits, kind="stable")
        ek[sl] = keys[sl][o]
        ev[sl] = vals[sl][o]
    return ek, ev


def _check(gpu, keys, nseg, seglen, begin=0, end=64):
    vals = np.arange(keys.size, dtype=np.int32)[::-1].copy()
    gk, gv = _sort(gpu, keys, vals, nseg, seglen, begin, end)
    ek, ev = _expect(keys, vals, nseg, seglen, begin, end)
    assert np.array_equal(gk, ek)
    assert np.array_equal(gv, ev)


def _doubles_as_keys(x):
    """the library's ordered_key (sort.hpp) of float64 values"""
    b = np.asarray(x, dtype=np.float64).view(np.uint64)
    neg = (b >> np.uint64(63)) == 1
    return np.where(neg, ~b, b | np.uint64(1 << 63)).astype(np.uint64)


@pytest.mark.parametrize("n", [2, 3, 64, 1000, 3700, LS_CAP])
def test_lds_sort_matches_stable_argsort(gpu, n):
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 2**64, n, dtype=np.uint64)
    keys[rng.integers(0, n, n // 3)] = keys[0]  # ties keep input order
    _check(gpu, keys, 1, n)


def test_lds_sort_on_a_bit_range_and_batched(gpu):
    rng = np.random.default_rng(7)
    keys = rng.integers(0, 2**64, 5 * 3000, dtype=np.uint64)
    _check(gpu, keys, 5, 3000, begin=4, end=20)  # garbage outside the bits is carried
    _check(gpu, keys, 5, 3000)


@pytest.mark.parametrize("n", [1 << 16, 100_000, 1 << 18, 1 << 19])
def test_sample_sort_matches_stable_argsort(gpu, n):
    rng = np.random.default_rng(n)
    x = rng.random(n)
    x[rng.integers(0, n, n // 4)] = x[5]           # a quarter of the keys one value
    x[rng.integers(0, n, n // 8)] = -0.0           # and the two zeros tie
    x[rng.integers(0, n, 100)] = 0.0
    _check(gpu, _doubles_as_keys(x), 1, n)


def test_sample_sort_sorted_reversed_and_constant_inputs(gpu):
    n = 1 << 18
    k = np.arange(n, dtype=np.uint64) * np.uint64(977)
    _check(gpu, k, 1, n)
    _check(gpu, k[::-1].copy(), 1, n)
    _check(gpu, np.full(n, 42, dtype=np.uint64), 1, n)


def test_sample_sort_batched_segments_and_bit_range(gpu):
    rng = np.random.default_rng(3)
    seglen = 212_736  # the unique-fitness count of a C5 generation
    keys = _doubles_as_keys(rng.random(2 * seglen))
    _check(gpu, keys, 2, seglen)
    raw = rng.integers(0, 2**64, 3 * 70_000, dtype=np.uint64)
    _check(gpu, raw, 3, 70_000, begin=8, end=56)  # 6 digits: sample sort on masked bits


def test_sample_sort_bucket_fallback(gpu):
    """Every key the splitter sample does not see lies between two sampled
    keys: one bucket holds nearly everything and is sorted by the
    workgroup-local radix fallback (sort.hip ss_bucket_kernel)."""
    n = 1 << 17
    stride = n // SS_SAMPLE  # (the sample sort's range starts at 2^16)
    i = np.arange(SS_SAMPLE, dtype=np.uint64)
    h = (i * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)
    sampled = i * np.uint64(stride) + (h >> np.uint64(8)) % np.uint64(stride)
    rng = np.random.default_rng(11)
    keys = (np.uint64(1000) * np.uint64(SS_SAMPLE)
            + rng.integers(0, 500, n, dtype=np.uint64))   # between sampled keys 999 and 1000
    keys[sampled.astype(np.int64)] = i * np.uint64(1000) * np.uint64(2)
    keys[sampled.astype(np.int64)[1000:]] += np.uint64(1 << 40)
    _check(gpu, keys, 1, n)


@pytest.mark.parametrize("n,end", [(1 << 20, 64), (300_000, 24), (LS_CAP + 1, 64), (20_000, 64)])
def test_radix_sort_paths_match_stable_argsort(gpu, n, end):
    rng = np.random.default_rng(end)
    keys = rng.integers(0, 2**64, n, dtype=np.uint64)
    keys[rng.integers(0, n, n // 5)] = keys[1]
    _check(gpu, keys, 1, n, 0, end)


def _seg_sort(gpu, keys, vals, starts, begin, end):
    import torch
    from deap_amd import _lib
    from deap_amd.device import Context
    fn = _lib.load().dm_test_seg_sort_pairs
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64]
    k = torch.from_numpy(keys.view(np.int64).copy()).to(gpu)
    v = torch.from_numpy(vals.copy()).to(gpu)
    st = torch.from_numpy(starts.astype(np.int32)).to(gpu)
    ctx = Context.get(gpu)
    _lib.check(fn(ctx.handle, ctypes.c_void_p(k.data_ptr()), ctypes.c_void_p(v.data_ptr()),
                  ctypes.c_void_p(st.data_ptr()), len(starts) - 1, begin, end, len(keys)),
               "dm_test_seg_sort_pairs")
    return k.cpu().numpy().view(np.uint64), v.cpu().numpy()


@pytest.mark.parametrize("end,cap", [(18, 8192), (64, LS_CAP)])
def test_segmented_lds_sort_matches_stable_argsort(gpu, end, cap):
    """Variable-length segments (the crowding distance's per-front sorts,
    nsga2.hip crowding_impl): empty, single, ragged and full-capacity ones;
    keys of <= 32 bits take the 8,192-pair kernel."""
    rng = np.random.default_rng(end)
    sizes = np.array([0, 1, 2, 33, cap, 700, 0, cap - 1, 3000, 5], dtype=np.int64)
    starts = np.concatenate([[0], np.cumsum(sizes)])
    n = int(starts[-1])
    hi = 1 << min(end, 63)
    keys = rng.integers(0, hi, n, dtype=np.uint64)
    keys[rng.integers(0, n, n // 4)] = keys[3]  # ties keep input order
    vals = np.arange(n, dtype=np.int32)[::-1].copy()
    gk, gv = _seg_sort(gpu, keys, vals, starts, 0, end)
    for a, b in zip(starts[:-1], starts[1:]):
        o = np.argsort(keys[a:b], kind="stable")
        assert np.array_equal(gk[a:b], keys[a:b][o])
        assert np.array_equal(gv[a:b], vals[a:b][o])


@pytest.mark.parametrize("end,cap", [(18, 8192), (64, LS_CAP)])
def test_segmented_lds_sort_oversized_segments_are_sorted(gpu, end, cap):
    """A segment over the LDS sort's capacity (the crowding sort's
    caller bound the largest front; a wrong bound must not leave a silently
    unsorted tail): sorted exactly through global memory instead."""
    rng = np.random.default_rng(100 + end)
    sizes = np.array([5, cap + 1, 0, 3 * cap + 17, 700], dtype=np.int64)
    starts = np.concatenate([[0], np.cumsum(sizes)])
    n = int(starts[-1])
    keys = rng.integers(0, 1 << min(end, 63), n, dtype=np.uint64)
    keys[rng.integers(0, n, n // 4)] = keys[2]
    vals = np.arange(n, dtype=np.int32)
    gk, gv = _seg_sort(gpu, keys, vals, starts, 0, end)
    for a, b in zip(starts[:-1], starts[1:]):
        o = np.argsort(keys[a:b], kind="stable")
        assert np.array_equal(gk[a:b], keys[a:b][o])
        assert np.array_equal(gv[a:b], vals[a:b][o])


@pytest.mark.parametrize("n", [1, 2048, 2049, 512 * 2048, 512 * 2048 + 1, 2048 * 2048,
                               2048 * 2048 + 5])
def test_device_scans_match_numpy(gpu, n):
    """Every scan form (one tile; reduce-then-scan with each block combining
    the aggregates before it, up to 512 tiles; with the aggregates scanned by
    one workgroup first, up to 2,048 tiles -- ADVICE r5; the block-sum form
    beyond), exclusive sum with its total and inclusive max."""
    import torch
    from deap_amd import _lib
    from deap_amd.device import Context
    fn = _lib.load().dm_test_scan_i32
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                   ctypes.c_void_p]
    rng = np.random.default_rng(n)
    x = rng.integers(-50, 100, n, dtype=np.int32)
    xi = torch.from_numpy(x).to(gpu)
    out = torch.empty_like(xi)
    tot = torch.zeros(1, dtype=torch.int32, device=gpu)
    ctx = Context.get(gpu)
    _lib.check(fn(ctx.handle, ctypes.c_void_p(xi.data_ptr()), ctypes.c_void_p(out.data_ptr()), n,
                  0, ctypes.c_void_p(tot.data_ptr())), "dm_test_scan_i32")
    ex = np.concatenate([[0], np.cumsum(x, dtype=np.int64)[:-1]]).astype(np.int32)
    assert np.array_equal(out.cpu().numpy(), ex)
    assert int(tot.cpu()[0]) == int(x.astype(np.int64).sum())
    _lib.check(fn(ctx.handle, ctypes.c_void_p(xi.data_ptr()), ctypes.c_void_p(out.data_ptr()), n,
                  1, None), "dm_test_scan_i32")
    assert np.array_equal(out.cpu().numpy(), np.maximum.accumulate(x))
