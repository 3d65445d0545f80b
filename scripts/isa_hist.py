"""Instruction mix of one kernel in a device assembly file (measurement aid).

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S \
      -I include structured_light_for_3d_model_replication_amd/csrc/slgpu.hip -o /tmp/slgpu.s
  python scripts/isa_hist.py /tmp/slgpu.s 'k_decodeILi11ELi0ELi322ELi1E' [--blocks]

Prints the kernel's register counts and its instructions by class (VALU /
SALU / VMEM / LDS / ...) and mnemonic; --blocks adds the static instruction
count of each basic block (the chunk-group loop is the largest block that
branches back).
"""
import collections
import re
import sys


def kernel_lines(path, key):
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        head = ln.split(";")[0].strip()
        if start is None and key in head and head.endswith(":") and not ln.startswith(("\t", ".")):
            start = i
        elif start is not None and ln.startswith(".Lfunc_end"):
            return lines[start:i], lines[i:i + 40]
    raise SystemExit(f"no kernel matching {key}")


def klass(m):
    if m.startswith("v_"):
        if m.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
            return "VALU-lane"
        return "VALU"
    if m.startswith("s_"):
        if m.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_sleep", "s_sched", "s_setprio")):
            return "SYNC"
        if m.startswith(("s_load", "s_buffer_load")):
            return "SMEM"
        if m.startswith(("s_cbranch", "s_branch")):
            return "BRANCH"
        return "SALU"
    if m.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "VMEM"
    if m.startswith("ds_"):
        return "LDS"
    return "OTHER"


def main():
    path, key = sys.argv[1], sys.argv[2]
    body, tail = kernel_lines(path, key)
    for ln in tail:
        if re.search(r"\.(num_vgpr|num_agpr|numbered_sgpr|private_seg_size),", ln):
            print(ln.strip())
    by_class, by_mn = collections.Counter(), collections.Counter()
    blocks, cur = [], ["entry", 0]
    for ln in body:
        s = ln.strip()
        if re.match(r"^\.?L?BB\d+_\d+:", s) or re.match(r"^\.LBB", s):
            blocks.append(tuple(cur))
            cur = [s.split(":")[0], 0]
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        m = s.split()[0]
        by_class[klass(m)] += 1
        by_mn[m] += 1
        cur[1] += 1
    blocks.append(tuple(cur))
    print("static instructions by class:", dict(by_class.most_common()))
    for m, n in by_mn.most_common(45):
        print(f"  {n:6d} {m}")
    if "--blocks" in sys.argv:
        for name, n in blocks:
            if n >= 20:
                print(f"  block {name}: {n}")


if __name__ == "__main__":
    main()
