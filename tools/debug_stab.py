"""Diagnostics: the forced-spill 768-d SQ8 case of tests/test_sq8_spill.py under second-level
variants (spill table sizes / bitset, first-level layouts and sizes, prefetch on / off); prints the
number of queries whose ids, distance bits or counters differ from the restatement's."""
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (runtime order)

    torch.cuda.is_available()
    import oracle
    from alayalite_amd import _native

    oracle.build()
    ext = _native._ext
    d, N, NQ, metric, order = 768, 20000, 24, 1, 2
    rng = np.random.default_rng(1000 + d + metric)
    centres = rng.standard_normal((64, d)).astype(np.float32)
    base = (centres[rng.integers(0, 64, N)] + 0.35 * rng.standard_normal((N, d))).astype(np.float32)
    queries = (centres[rng.integers(0, 64, NQ)] + 0.35 * rng.standard_normal((NQ, d))).astype(np.float32)
    g = ext.Graph.build(base, metric, 32, 100, 8, 100)
    mn, mx = ext.sq8_train(base)
    codes = ext.sq8_encode(base, mn, mx, 8)
    l0, levels, off, ue, ep, ur, _ = g.arrays()
    view = oracle.IndexView(base, l0, levels, off, ue, ur, ep, metric=metric, sq8=(codes, mn, mx, order))
    for ef in (40, 340):
        expect = [view.search(q, 10, ef, with_counters=True) for q in queries]
        for st, vm, hl, fl, w in itertools.product(["d", "0", "16", "6"], [1, 2], [7, 10], ["0", "1"], ["1", "4"]):
            os.environ.pop("ALAYA_SPILL_TABLE", None)
            if st != "d":
                os.environ["ALAYA_SPILL_TABLE"] = st
            os.environ["ALAYA_SPILL_FLAGS"] = fl
            os.environ["ALAYA_SEARCH_WAVES"] = w
            dev = ext.DeviceIndex(0)
            dev.set_base(base, metric)
            dev.set_graph(g)
            dev.set_sq8(codes, mn, mx, order)
            dev.set_hash_log2(hl)
            dev.set_visited_mode(vm)
            ids, dd, cc = dev.search_sq8(queries, 10, ef, 0)
            bad = [i for i in range(NQ) if not (np.array_equal(ids[i], expect[i][0]) and tuple(cc[i]) == tuple(expect[i][2]))]
            first = "" if not bad else f" first q{bad[0]}: n_dist {cc[bad[0]][0]} vs {expect[bad[0]][2][0]}"
            print(f"ef {ef} table {st:>2} visited {vm} log2 {hl:2d} flags {fl} waves {w}: {len(bad)} bad{first}", flush=True)


if __name__ == "__main__":
    main()
