"""Resolve the preprocessor knobs of the RT kernel sources that no shipped
kernel image varies ("prune the rejected knobs").

Every #if / #ifdef / #ifndef chain of the given device-only sources is
instrumented with marker lines, each shipped image's compile line is run
through the device preprocessor (hipcc -E --cuda-device-only), and a chain
that takes the same branch in every image that reaches it is replaced by that
branch.  Chains that differ between images (RT_INSTRUMENT, RT_STAMPS, the
deep / flat / compact images) stay.  The caller then checks that the shipped
images rebuild bit-identical.

    python scripts/prune_knobs.py            # dry run: report
    python scripts/prune_knobs.py --write    # rewrite the sources
"""
from __future__ import annotations

import argparse
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "skybox_rt_amd", "csrc")
KDIR = os.path.join(CSRC, "kernels")
FILES = ["rt_trace.h", "rt_kernel.hip", "pt_kernel.hip"]

# the shipped images' defines (skybox_rt_amd/csrc/Makefile: IMAGES and diag)
RT_BASE = "-DRT_ONLY_BVH4H=1"
RT_DEFS = RT_BASE + " -DRT_BLOCK_THREADS=128"
BVH_DEFS = RT_BASE + " -DRT_BLOCK_THREADS=256 -DRT_BVH_WALK=1"
PT_DEFS = "-DRT_ONLY_BVH4H=1 -DRT_PUSH_UNCOND=1 -DRT_LAZY_TASK_ARGS=0 -DVX_ROWS_GATE=0"
FLAT_DEFS = "-DRT_FLAT=1 -DRT_BLOCK_THREADS=512"
# (source, defines) of every shipped image and the diagnostic stamp images
CONFIGS = []
for inst in ("", " -DRT_INSTRUMENT"):
    CONFIGS += [
        ("rt_kernel.hip", RT_DEFS + inst),
        ("rt_kernel.hip", BVH_DEFS + inst),
        ("rt_kernel.hip", "-DRT_MAX_STACK=32" + inst),
        ("rt_kernel.hip", FLAT_DEFS + inst),
        ("rt_kernel.hip", RT_DEFS + " -DRT_PATHQ=1" + inst),
        ("rt_kernel.hip", RT_BASE + " -DRT_BLOCK_THREADS=64 -DRT_STAMPS" + inst),
        ("rt_kernel.hip", RT_BASE + " -DRT_BLOCK_THREADS=64 -DRT_BVH_WALK=1 -DRT_STAMPS" + inst),
        ("rt_kernel.hip", FLAT_DEFS + " -DRT_STAMPS" + inst),
        ("pt_kernel.hip", PT_DEFS + inst),
        ("pt_kernel.hip", "-DRT_MAX_STACK=32" + inst),
        ("pt_kernel.hip", "-DPT_MODE=0" + inst),
        ("pt_kernel.hip", PT_DEFS + " -DPT_MODE=2 -DPT_PAIR=0" + inst),
        ("pt_kernel.hip", PT_DEFS + " -DRT_STAMPS -DRT_TRACE_CYCLES" + inst),
    ]

DIRECTIVE = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b")


def logical_lines(lines):
    """[(first, last)] physical line ranges of each logical line"""
    out, i = [], 0
    while i < len(lines):
        j = i
        while lines[j].rstrip("\n").endswith("\\") and j + 1 < len(lines):
            j += 1
        out.append((i, j))
        i = j + 1
    return out


def parse(lines):
    """conditional chains: list of dicts {branches: [(dir_line, body_first, body_last)], end}"""
    chains, stack = [], []
    for first, last in logical_lines(lines):
        m = DIRECTIVE.match(lines[first])
        if not m:
            continue
        kind = m.group(1)
        if kind in ("if", "ifdef", "ifndef"):
            stack.append({"branches": [[first, last + 1, None]], "end": None})
        elif kind in ("elif", "else"):
            ch = stack[-1]
            ch["branches"][-1][2] = first - 1
            ch["branches"].append([first, last + 1, None])
        else:
            ch = stack.pop()
            ch["branches"][-1][2] = first - 1
            ch["end"] = first
            chains.append(ch)
    assert not stack, "unbalanced conditionals"
    return chains


def instrument(lines, tag):
    """marker after every branch directive and before every chain"""
    chains = parse(lines)
    after, before = {}, {}
    for ci, ch in enumerate(chains):
        before[ch["branches"][0][0]] = f"PRUNEMARK_{tag}_R{ci}\n"
        for bi, (d, b0, b1) in enumerate(ch["branches"]):
            after[b0 - 1] = f"PRUNEMARK_{tag}_B{ci}_{bi}\n"
    out = []
    for i, ln in enumerate(lines):
        if i in before:
            out.append(before[i])
        out.append(ln)
        if i in after:
            out.append(after[i])
    return out, chains


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--write", action="store_true")
    args = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="prune_")
    tk = os.path.join(tmp, "kernels")
    shutil.copytree(KDIR, tk)
    src = {f: open(os.path.join(KDIR, f)).readlines() for f in FILES}
    chains = {}
    for f in FILES:
        tag = re.sub(r"\W", "_", f)
        inst, chains[f] = instrument(src[f], tag)
        with open(os.path.join(tk, f), "w") as fh:
            fh.writelines(inst)
    seen = []
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    for source, defs in CONFIGS:
        cmd = [hipcc, "-E", "--cuda-device-only", "--offload-arch=gfx950", "-std=c++17",
               "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(CSRC, "runtime"),
               "-I" + os.path.join(CSRC, "app"), "-I" + tk] + defs.split() + [os.path.join(tk, source)]
        out = subprocess.run(cmd, capture_output=True, text=True)
        if out.returncode != 0:
            sys.exit(out.stderr)
        seen.append(set(re.findall(r"PRUNEMARK_\w+", out.stdout)))
    total_kept = 0
    for f in FILES:
        tag = re.sub(r"\W", "_", f)
        lines = src[f]
        drop = set()      # physical lines to delete
        resolved = 0
        for ci, ch in enumerate(chains[f]):
            reach = [s for s in seen if f"PRUNEMARK_{tag}_R{ci}" in s]
            if not reach:
                continue  # inside a dead region: goes with its parent
            taken = set()
            for s in reach:
                bs = [bi for bi in range(len(ch["branches"])) if f"PRUNEMARK_{tag}_B{ci}_{bi}" in s]
                taken.add(bs[0] if bs else -1)
            if len(taken) != 1:
                continue
            keep = taken.pop()
            resolved += 1
            for bi, (d, b0, b1) in enumerate(ch["branches"]):
                # the directive line(s)
                nxt = ch["branches"][bi + 1][0] if bi + 1 < len(ch["branches"]) else ch["end"]
                for i in range(d, b0):
                    drop.add(i)
                if bi != keep:
                    for i in range(b0, nxt):
                        drop.add(i)
            drop.add(ch["end"])
        kept = len(chains[f]) - resolved
        total_kept += kept
        print(f"{f}: {len(chains[f])} chains, {resolved} resolved, {kept} kept")
        if args.write:
            with open(os.path.join(KDIR, f), "w") as fh:
                fh.writelines(ln for i, ln in enumerate(lines) if i not in drop)
    shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
