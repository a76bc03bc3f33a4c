"""ISA guards on the search kernels (CPU-only: hipcc cross-compiles gfx950 to assembly here).

tools/isa_census.py finds each hnsw_search_kernel instantiation's expansion loops (the depth-2 loops
that probe the LDS visited table and gather rows) and counts SGPR spill restores inside them.  A
restore there runs once per expansion; round 3 took the d = 960 kernel (the headline) from 108 to 0
and the d = 128 kernel from 2 to 0.  These tests keep it that way, and keep the
register budgets the residency policy was measured with."""

import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"),
                                reason="needs hipcc to compile the kernels to assembly")


@pytest.fixture(scope="module")
def census():
    import isa_census as ic

    asm = ic.compile_asm(ic.SRC, [])
    rows = {}
    for name, body in ic.split_functions(asm).items():
        if "hnsw_search_kernel" in name:
            r = ic.census(name, body)
            r.update(ic.resource_comments(asm, name))
            rows[r["kernel"]] = r
    return rows


@pytest.mark.parametrize("chunks", [4, 8, 16, 24, 30, 32])
@pytest.mark.parametrize("metric", ["l2", "ip"])
def test_fixed_d_f32_expansion_loops_restore_no_spilled_sgpr(census, metric, chunks):
    r = census[f"{metric} chunks={chunks} stamp=0 space=f32"]
    assert r["expansion_loops"], "no expansion loop found"
    assert r["restores_in_expansion_loops"] == 0, r["expansion_loops"]


# The AVX-512-order SQ8 kernels carry the spill table (round 4: flush, bucket prefetch, bitset third
# level), whose uniform state costs SGPR restores per expansion -- 10-21 v_readlane against ~12k
# cycles per expansion at config 5 (measured on this image's hipcc: 21 in config 5's 768-d IP
# kernel since the paired lane loops, 10-17 in the others).  The AVX2-order kernels keep the bitset
# (2-6 restores).  Budgets are the measured maxima plus a small margin, so a regression shows up
# here first.
SQ8_RESTORE_BUDGET = {"sq8-avx512": 23, "sq8-avx2": 6}
# scratch bytes the AVX-512-order SQ8 kernels may use (held to 128 VGPRs: a value or two live across
# the query loop, stored at kernel entry and loaded after it -- never inside an expansion)
SQ8_SCRATCH_BYTES = {"ip chunks=24": 12, "l2 chunks=24": 0, "ip chunks=30": 28, "l2 chunks=30": 12}


@pytest.mark.parametrize("space", ["sq8-avx512", "sq8-avx2"])
@pytest.mark.parametrize("chunks", [4, 24, 30])
def test_sq8_expansion_loops_restore_few_spilled_sgpr(census, space, chunks):
    r = census[f"ip chunks={chunks} stamp=0 space={space}"]
    assert r["expansion_loops"], "no expansion loop found"
    assert r["restores_in_expansion_loops"] <= SQ8_RESTORE_BUDGET[space], r["expansion_loops"]


def test_register_budgets(census):
    # no scratch traffic per expansion in any search kernel, and no scratch at all outside the
    # AVX-512-order SQ8 kernels -- those are held to 128 VGPRs (4 waves per SIMD; config 5's 768-d IP
    # kernel needs 129), which costs a value or two live across the query loop: stored at kernel
    # entry, loaded after the loop.  The d = 128 kernels stay at >= 4 waves per SIMD (the
    # residency cap is 4).
    for k, r in census.items():
        if "stamp=0" in k:  # (the stamped kernels are diagnostics builds)
            assert r["scratch_ops_in_expansion_loops"] == 0, k
        if "sq8-avx512" in k and "chunks=0" not in k and "stamp=0" in k:
            budget = SQ8_SCRATCH_BYTES.get(k.split(" stamp")[0], 0)
            # exactly the measured bytes: a new spilled value shows up here even outside the loops
            assert r.get("ScratchSize", 0) == budget and r["scratch_ops_total"] <= 8, (k, r.get("ScratchSize"))
        elif "stamp=0" in k:
            assert r.get("ScratchSize", 0) == 0, k
    assert census["ip chunks=24 stamp=0 space=sq8-avx512"]["NumVgprs"] <= 128
    for m in ("l2", "ip"):
        assert census[f"{m} chunks=4 stamp=0 space=f32"]["Occupancy"] >= 4


# SGPR restores per expansion in the helper kernels: measured 3 (f32), 40 / 48 (SQ8 IP / L2, 768-d)
HELPER_RESTORE_BUDGET = {"chunks=4": 5, "chunks=8": 5, "chunks=24 sq8": 50}


@pytest.mark.parametrize("kernel", ["l2 chunks=4 stamp=4 space=f32", "ip chunks=4 stamp=4 space=f32",
                                    "l2 chunks=8 stamp=4 space=f32",
                                    "ip chunks=24 stamp=4 space=sq8-avx512", "l2 chunks=24 stamp=4 space=sq8-avx512"])
def test_helper_kernels_keep_the_expansion_loop_clean(census, kernel):
    """The distance-helper kernels (kMode 4: memo lookups in the expansion, the help loop after it) for
    the SIFT shape (d = 128 / 256) and config 5 (768-d SQ8): no scratch traffic per expansion, few
    SGPR restores, and the residency the searches were measured with."""
    r = census[kernel]
    assert r["expansion_loops"], "no expansion loop found"
    # since the helpers retire their requests before clearing the memo (round 6), config 5's 768-d IP
    # kernel reloads one value on the path of an expansion's second row pass (more than 16 fresh rows,
    # rare at ~6.3 per expansion); the 768-d L2 one (no benchmark shape) two
    budget = 1 if kernel.startswith("ip chunks=24") else (2 if kernel.startswith("l2 chunks=24") else 0)
    assert r["scratch_ops_in_expansion_loops"] <= budget, r
    assert r["restores_in_expansion_loops"] <= HELPER_RESTORE_BUDGET[kernel.split(" stamp")[0].split(" ")[1] + (
        " sq8" if "sq8" in kernel else "")], r
    assert r["Occupancy"] >= (3 if "chunks=8" in kernel else 4), r


@pytest.mark.parametrize("kernel", ["l2 chunks=30 stamp=8 space=f32", "ip chunks=30 stamp=8 space=f32",
                                    "l2 chunks=24 stamp=8 space=f32"])
def test_two_waves_wide_row_kernels(census, kernel):
    """kMode 8: the wide-row f32 kernels at two waves per SIMD (one row per lane group) -- within
    256 registers, no scratch, and the headline's one-wave kernel keeps its 24 rows per pass."""
    r = census[kernel]
    assert r["Occupancy"] >= 2 and r.get("ScratchSize", 0) == 0, r
    assert r["restores_in_expansion_loops"] == 0, r
    one = census[kernel.replace("stamp=8", "stamp=0")]
    assert one["Occupancy"] == 1 and one.get("ScratchSize", 0) == 0, one
