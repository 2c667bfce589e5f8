"""Static check of the hand-written LDS reads: compiles HIP sources for gfx950
to assembly (device only, the Makefile's flags) and, in every kernel, follows
each inline-asm ds_read to the s_waitcnt that completes it, flagging any
instruction in between that touches the read's destination registers.

An inline-asm read's result arrives asynchronously, but the compiler takes
the destination as written when the asm statement issues; if it deems the
value dead (a last iteration's prefetch) or copies it early, it may recycle
the register while the return is still in flight -- round 5's
crossnet_dw_w4_kernel recycled one for a global_load_lds address and faulted.
Waits counted as lgkmcnt(N) complete a read once N later LDS/SMEM operations
have issued after it.  Branches end the scan (loop-carried reads are covered
by the "+v" ties on the waits themselves).

usage: python tools/lds_hazard_scan.py [csrc/file.hip ...]   (exit 1 on a hazard)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "deeprec-1_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "--offload-arch=gfx950",
         "--cuda-device-only", "-S", "-I" + CSRC, "-I" + os.path.join(ROOT, "include")]


def _regs(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def scan_asm(text):
    """[(kernel, read, offending instruction)] over an assembly listing."""
    found = []
    for name in re.findall(r"^(_Z\w+):", text, re.M):
        i = text.index(name + ":")
        j = text.index(".Lfunc_end", i)
        ins, in_asm = [], False
        for line in text[i:j].splitlines():
            line = line.strip()
            if line.startswith(";;#ASMSTART"):
                in_asm = True
            elif line.startswith(";;#ASMEND"):
                in_asm = False
            elif line and not line.startswith((";", ".")) and not line.endswith(":"):
                ins.append((line, in_asm))
        for k, (line, a) in enumerate(ins):
            if not (a and line.startswith("ds_read")):
                continue
            dst = _regs(line.split()[1].rstrip(","))
            later = 0
            for l2, _ in ins[k + 1:]:
                m = re.search(r"lgkmcnt\((\d+)\)", l2)
                if l2.startswith("s_waitcnt") and m and later >= int(m.group(1)):
                    break
                if l2.startswith(("s_cbranch", "s_branch", "s_endpgm", "s_setpc")):
                    break
                if l2.startswith(("ds_", "s_load", "s_buffer_load")):
                    later += 1
                ops = [t.rstrip(",") for t in l2.split()[1:]]
                if any(_regs(t) & dst for t in ops):
                    found.append((name, line, l2))
                    break
    return found


def scan_file(path):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + [path, "-o", out], check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        with open(out) as f:
            return scan_asm(f.read())


def main(argv):
    files = argv or [os.path.join(CSRC, f) for f in ("interact.hip", "grad_rows.hip", "pool.hip")]
    bad = 0
    for path in files:
        hits = scan_file(path)
        print("%s: %d hazard(s)" % (os.path.basename(path), len(hits)))
        for name, r, o in hits[:10]:
            print("  %s\n    %s\n    %s" % (name, r, o))
        bad += len(hits)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
