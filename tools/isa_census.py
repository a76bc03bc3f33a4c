"""ISA census of the search kernels: registers, SGPR spills, and where the spill traffic sits.

Compiles csrc/search_kernels.hip for gfx950 to assembly (device only, same flags as _build.py) and,
for every hnsw_search_kernel instantiation, reports
  * VGPRs / AGPRs / SGPRs and occupancy (the compiler's own comments),
  * SGPR spill slots (``v_writelane`` into the "SGPR spill to VGPR lane" registers) and the spill
    restores (``v_readlane`` from them),
  * how many of those restores sit inside the expansion loop -- the per-query ``while (cur < size)``
    loop: a depth-2 loop (LLVM's "Loop: Header=..." block comments) that both probes the LDS
    visited table and gathers rows -- versus the per-query setup / teardown around it.
A restore outside the expansion loop runs a handful of times per query; one inside it runs once
per expansion (~90 times per SIFT query at ef 70).

usage: python tools/isa_census.py [--out profiles/r03/isa/search_isa_census.json] [--filter 'Li4E']
"""

from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "alayalite_amd", "csrc", "search_kernels.hip")


def compile_asm(src: str, extra: list[str]) -> str:
    out = os.path.join(tempfile.mkdtemp(prefix="isa_"), "k.s")
    cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           f"-I{os.path.join(ROOT, 'include')}", "--cuda-device-only", "-S", src, "-o", out] + extra
    subprocess.run(cmd, check=True)
    with open(out) as f:
        return f.read()


def demangle(name: str) -> str:
    m = re.search(r"hnsw_search_kernelILb(\d)ELi(\d+)EL[bi](\d)ELi(\d)E", name)
    if not m:
        return name
    ip, chunks, stamp, space = m.groups()
    return f"{'ip' if ip == '1' else 'l2'} chunks={chunks} stamp={stamp} space={['f32', 'sq8-avx2', 'sq8-avx512'][int(space)]}"


def split_functions(asm: str) -> dict[str, list[str]]:
    lines = asm.split("\n")
    funcs, cur, body = {}, None, []
    for ln in lines:
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if ln.startswith(".Lfunc_end"):
                funcs[cur] = body
                cur = None
            else:
                body.append(ln)
    return funcs


def resource_comments(asm: str, name: str) -> dict:
    # the per-kernel comment block follows the function body: "; NumVgprs: N" etc.
    i = asm.find(f".Lfunc_end")
    start = asm.find(name + ":")
    block = asm[start:]
    end = block.find("; Occupancy:")
    block = block[: block.find("\n", end) + 1] if end >= 0 else block[:0]
    out = {}
    for key in ("TotalNumSgprs", "NumVgprs", "NumAgprs", "TotalNumVgprs", "ScratchSize", "Occupancy"):
        m = re.search(rf"; {key}: (\d+)", block)
        if m:
            out[key] = int(m.group(1))
    del i
    return out


def census(name: str, body: list[str]) -> dict:
    spill_regs = set()
    for ln in body:
        m = re.search(r"implicit-def: \$vgpr(\d+) : SGPR spill to VGPR lane", ln)
        if m:
            spill_regs.add(f"v{m.group(1)}")
    # Loop nesting from LLVM's block comments: a loop header lists its ancestors ("Parent Loop H
    # Depth=d") before "This (Inner) Loop Header"; any other block names only its innermost loop
    # ("in Loop: Header=H").  A block's chain = ancestors(innermost) + innermost.
    parents: dict[str, list[str]] = {}
    depth: dict[str, int] = {}
    insts: list[tuple[tuple[str, ...], str]] = []
    chain: tuple[str, ...] = ()
    label, pend = None, []
    for ln in body:
        s = ln.strip()
        m = re.match(r"^(?:\.L(BB\S+):|; %(bb\.\d+):)", s)
        if m:
            label = m.group(1) or m.group(2)
            pend = []
            chain = ()
            m2 = re.search(r"in Loop: Header=(BB\S+) Depth=(\d+)", s)
            if m2:
                chain = tuple(parents.get(m2.group(1), [])) + (m2.group(1),)
            m2 = re.search(r"Parent Loop (BB\S+) Depth=(\d+)", s)
            if m2:
                pend.append(m2.group(1))
                depth[m2.group(1)] = int(m2.group(2))
            m2 = re.search(r"This (?:Inner )?Loop Header: Depth=(\d+)", s)
            if m2:
                parents[label] = list(pend)
                depth[label] = int(m2.group(1))
                chain = tuple(pend) + (label,)
            continue
        if s.startswith(";"):
            m2 = re.search(r"Parent Loop (BB\S+) Depth=(\d+)", s)
            if m2:
                pend.append(m2.group(1))
                depth[m2.group(1)] = int(m2.group(2))
            m2 = re.search(r"This (?:Inner )?Loop Header: Depth=(\d+)", s)
            if m2 and label:
                parents[label] = list(pend)
                depth[label] = int(m2.group(1))
                chain = tuple(pend) + (label,)
            continue
        if not s or s.startswith("."):
            continue
        insts.append((chain, s))

    def is_restore(s: str) -> bool:
        m = re.match(r"v_readlane_b32 s\d+, (v\d+), (\d+)$", s)
        return bool(m) and m.group(1) in spill_regs

    def is_spill(s: str) -> bool:
        m = re.match(r"v_writelane_b32 (v\d+), s\d+, (\d+)$", s)
        return bool(m) and m.group(1) in spill_regs

    # expansion loops: depth-2 loops (inside the persistent query loop) that both insert into the
    # LDS visited table (ds_cmpst / ds_cmpswap) and gather rows (global_load_dword*); loop
    # unswitching can leave more than one copy
    loops = {}
    for h, d in depth.items():
        if d != 2:
            continue
        ins = [s for c, s in insts if h in c]
        if any(s.startswith(("ds_cmpst", "ds_cmpswap")) for s in ins) and any(s.startswith("global_load_dword") for s in ins):
            loops[h] = {
                "insts": len(ins),
                "restores": sum(1 for s in ins if is_restore(s)),
                "spill_stores": sum(1 for s in ins if is_spill(s)),
                "scratch_ops": sum(1 for s in ins if s.startswith(("scratch_", "buffer_store", "buffer_load"))),
                "valu": sum(1 for s in ins if s.startswith("v_")),
                "salu": sum(1 for s in ins if s.startswith("s_") and not s.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch"))),
            }
    return {
        "kernel": demangle(name),
        "spill_vgprs": sorted(spill_regs),
        "spill_slots": len({re.match(r"v_writelane_b32 (v\d+), s\d+, (\d+)", s).groups()
                            for _, s in insts if is_spill(s)}),
        "restores_total": sum(1 for _, s in insts if is_restore(s)),
        "expansion_loops": loops,
        "restores_in_expansion_loops": sum(v["restores"] for v in loops.values()),
        "scratch_ops_total": sum(1 for _, s in insts if s.startswith(("scratch_", "buffer_store", "buffer_load"))),
        "scratch_ops_in_expansion_loops": sum(v["scratch_ops"] for v in loops.values()),
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--filter", default="hnsw_search_kernel")
    ap.add_argument("--extra", default="", help="extra hipcc flags (e.g. -DALAYA_...)")
    args = ap.parse_args()
    asm = compile_asm(SRC, args.extra.split())
    rows = []
    for name, body in split_functions(asm).items():
        if "hnsw_search_kernel" not in name or args.filter not in name:
            continue
        r = census(name, body)
        r.update(resource_comments(asm, name))
        rows.append(r)
    for r in rows:
        print(f"{r['kernel']:<44} scratch {r.get('ScratchSize', '?'):>3} sgpr {r.get('TotalNumSgprs', '?'):>3} vgpr {r.get('NumVgprs', '?'):>3} "
              f"occ {r.get('Occupancy', '?')}  spill slots {r['spill_slots']:>2}  restores {r['restores_total']:>3} "
              f"(in expansion loops: {r['restores_in_expansion_loops']}; loops {len(r['expansion_loops'])}, "
              f"scratch ops {r['scratch_ops_total']} / in loops {r['scratch_ops_in_expansion_loops']}, "
              f"insts {sum(v['insts'] for v in r['expansion_loops'].values())})")
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
