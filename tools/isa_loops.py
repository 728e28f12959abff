"""Loop summary of one kernel of the HIP library's gfx950 code object.

usage: python tools/isa_loops.py [--lib path/to/liblgs_hip.so] [--min-len 100] MANGLED_PREFIX
e.g.   python tools/isa_loops.py _ZN3lgs17klein_mfma_kernelIsLi32ELb0ELb1ELb0E

Disassembles the code object (llvm-objdump --offloading, then -d), finds every
backward branch of the kernel and prints, per loop (instruction range of the
listing): its length and counts of fp64 FMAs, global stores / loads, vmcnt waits,
scratch (spill) accesses, MFMAs, barriers and calls.  Round 4 used it to find the
near-field loop's only `s_waitcnt vmcnt(0)` -- the reload of a spilled constant,
which also waited for every coordinate's stores (performance log).
--dump FILE writes the kernel's listing."""
import argparse
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def listing(lib, prefix):
    with tempfile.TemporaryDirectory() as td:
        tgt = os.path.join(td, "lib.so")
        os.symlink(os.path.abspath(lib), tgt)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", tgt], cwd=td, check=True, stdout=subprocess.DEVNULL)
        co = sorted(f for f in os.listdir(td) if f.endswith("gfx950"))[0]
        txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", os.path.join(td, co)],
                             capture_output=True, text=True, check=True).stdout
    lines = txt.split("\n")
    st = [i for i, l in enumerate(lines) if re.match(r"^[0-9a-f]+ <" + re.escape(prefix), l)]
    if not st:
        raise SystemExit(f"no kernel {prefix}")
    base = int(lines[st[0]].split()[0], 16)
    e = st[0] + 1
    while e < len(lines) and not re.match(r"^[0-9a-f]+ <", lines[e]):
        e += 1
    return base, lines[st[0]:e]


def loops(base, K, min_len):
    pos = {}
    for i, l in enumerate(K):
        m = re.search(r"//\s*([0-9A-F]{12}):", l)
        if m:
            pos[int(m.group(1), 16)] = i
    out = []
    for i, l in enumerate(K):
        if not re.search(r"s_(cbranch_\w+|branch)\s", l):
            continue
        t = re.search(r"<[^>+]+\+0x([0-9a-f]+)>", l)
        if not t:
            continue
        ta = base + int(t.group(1), 16)
        if ta in pos and pos[ta] < i and i - pos[ta] >= min_len:
            body = K[pos[ta]:i + 1]
            c = lambda s: sum(s in x for x in body)
            out.append(dict(first=pos[ta], last=i, length=len(body), fma_f64=c("v_fma_f64"),
                            stores=c("global_store"), loads=c("global_load"),
                            vmcnt_waits=sum(("s_waitcnt" in x and "vmcnt" in x) for x in body),
                            scratch=c("scratch_"), mfma=c("v_mfma"), barriers=c("s_barrier"),
                            calls=c("s_swappc")))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--lib", default=os.path.join(REPO, "lattice-gaussian-mcmc_amd", "lgs_amd", "_lib", "liblgs_hip.so"))
    ap.add_argument("--min-len", type=int, default=100)
    ap.add_argument("--dump", default="")
    args = ap.parse_args()
    base, K = listing(args.lib, args.prefix)
    if args.dump:
        with open(args.dump, "w") as f:
            f.write("\n".join(K))
    for lp in loops(base, K, args.min_len):
        print(" ".join(f"{k} {v}" for k, v in lp.items()))
