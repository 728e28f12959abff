"""Code-object resource summary of the built library (gfx950): per kernel the
VGPR / AGPR / SGPR counts, spills, scratch (private segment) and LDS (group
segment) bytes, and the waves per SIMD those allow (512 unified VGPRs per lane
per SIMD, 160 KB LDS per CU).

    python tools/co_resources.py [--lib PATH] [--filter klein] [--json OUT]

Unbundles the device code objects with clang-offload-bundler into a temporary
directory and parses `llvm-readelf --notes` (AMDGPU HSA metadata, YAML-like).
"""
import argparse
import glob
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("agpr_count", "vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
          "private_segment_fixed_size", "group_segment_fixed_size", "max_flat_workgroup_size")


def kernels(lib):
    out = []
    with tempfile.TemporaryDirectory() as td:
        tgt = os.path.join(td, "lib.so")
        os.symlink(os.path.abspath(lib), tgt)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", tgt], cwd=td, check=True,
                       stdout=subprocess.DEVNULL)
        for co in sorted(glob.glob(os.path.join(td, "lib.so.*gfx950"))):
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True,
                                   text=True, check=True).stdout
            # kernel entries are list items "  - .agpr_count: ..." up to the next one
            for blk in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
                blk = ".agpr_count:" + blk
                rec = {}
                m = re.search(r"\.name:\s+(\S+)", blk)
                if not m:
                    continue
                rec["name"] = m.group(1)
                for f in FIELDS:
                    mm = re.search(r"\." + f + r":\s+(\d+)", blk)
                    if mm:
                        rec[f] = int(mm.group(1))
                out.append(rec)
    return out


def waves_per_simd(r, block=256):
    # .vgpr_count is the unified total (arch VGPRs + AGPRs, gfx90a+): 512 per lane per
    # SIMD, allocation granule 8
    v = r.get("vgpr_count", 0)
    vg = 512 // max(8, -(-v // 8) * 8) if v else 8
    lds = r.get("group_segment_fixed_size", 0)
    wpb = max(1, -(-r.get("max_flat_workgroup_size", block) // 64))
    blocks_lds = (160 * 1024) // lds if lds else 32
    lg = blocks_lds * wpb // 4
    return min(vg, lg, 8), vg, lg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(REPO, "lattice-gaussian-mcmc_amd/lgs_amd/_lib/liblgs_hip.so"))
    ap.add_argument("--filter", default="")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    ks = [k for k in kernels(a.lib) if a.filter in k["name"]]
    bid = hashlib.sha256(open(a.lib, "rb").read()).hexdigest()[:16]
    rows = []
    for k in ks:
        w, wv, wl = waves_per_simd(k)
        k.update(waves_per_simd=w, waves_by_vgpr=wv, waves_by_lds=wl)
        rows.append(k)
        print(f"{k['name'][:90]:90s} vgpr {k.get('vgpr_count')} agpr {k.get('agpr_count')} "
              f"sgpr {k.get('sgpr_count')} spill v{k.get('vgpr_spill_count')}/s{k.get('sgpr_spill_count')} "
              f"scratch {k.get('private_segment_fixed_size')} lds {k.get('group_segment_fixed_size')} "
              f"waves/SIMD {w} (vgpr {wv}, lds {wl})")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"build_id": bid, "lib": os.path.relpath(a.lib, REPO), "kernels": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
