#!/usr/bin/env python3
"""VALU / SALU / LDS instruction counts of the fused kernel's phases from its ISA (the per-phase table
of DESIGN.md §5.3, with scripts/phase_stats.py's iteration counts).  The diagnostic build's s_memtime
marks (PT_PHASE_STATS) delimit the phases; backward branches delimit the loops.
Make the assembly first:
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \\
        -DPT_PHASE_STATS=1 --cuda-device-only -S -o diag.s brown-cs2240-path-tracer_amd/csrc/pt_wavefront.hip
usage: isa_phases.py diag.s [EXT=1|0]"""
import re
import sys

PHASES = ["load", "phase1", "replay", "path logic", "append"]


def body(path, name):
    lines = open(path).read().split("\n")
    st = [i for i, l in enumerate(lines) if l.startswith(name + ":")][0]
    end = [i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end")][0]
    return lines[st:end]


def main():
    ext = (sys.argv[2] if len(sys.argv) > 2 else "1") == "1"
    inst = ("ILb1" if ext else "ILb0") + "ELb1ELb1ELb0ELb0E"  # <EXT, LDS, rcp, !COUNT, !GEN>: the bench's instances
    name = "_ZN2pt12k_wf_step_bf" + inst + "EEvNS_9SceneViewENS_11FrameParamsENS_9WfBuffersEiPNS_8CountersEijjjjb"
    seq = []
    for l in body(sys.argv[1], name):
        if re.match(r"^\.LBB\S+:", l):
            seq.append(("L", l.split(":")[0]))
        elif l.startswith("\t") and not l.strip().startswith((".", ";")):
            seq.append(("I", l.strip()))
    pos, k = {}, 0
    for t, x in seq:
        if t == "L":
            pos[x] = k
        else:
            k += 1
    ins = [x for t, x in seq if t == "I"]
    mt = [i for i, l in enumerate(ins) if l.startswith("s_memtime")]

    def counts(seg):
        return (sum(1 for x in seg if x.startswith("v_")), sum(1 for x in seg if x.startswith("s_")),
                sum(1 for x in seg if x.startswith("ds_")))
    print(f"{'extension' if ext else 'shadow'} instance: phases (static counts between the s_memtime marks)")
    for j, ph in enumerate(PHASES):
        v, s, d = counts(ins[mt[j]:mt[j + 1]])
        print(f"  {ph:11s} instrs {mt[j + 1] - mt[j]:5d}  valu {v:4d}  salu {s:4d}  lds {d:3d}")
    print("loops (backward branches; nested loops include their inner loops):")
    for i, l in enumerate(ins):
        m = re.match(r"s_cbranch_\w+ (\.LBB\S+)|s_branch (\.LBB\S+)", l)
        if m:
            tgt = m.group(1) or m.group(2)
            if pos[tgt] <= i and mt[0] <= pos[tgt] and i < mt[-1]:
                ph = max(j for j in range(len(PHASES)) if mt[j] <= pos[tgt])
                v, s, d = counts(ins[pos[tgt]:i + 1])
                print(f"  [{PHASES[ph]}] {pos[tgt]}..{i}: valu {v} salu {s} lds {d}")


if __name__ == "__main__":
    main()
