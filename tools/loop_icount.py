#!/usr/bin/env python3
"""Static instruction count of every loop in each kernel of the device assembly (hipcc -S).

Usage: python3 tools/loop_icount.py [kernels.s]   (default: compiles hpmpc_kernels.hip to /tmp)
A loop = blocks tagged '; in Loop: Header=BBx_y' plus the header block.  Counts include both sides
of every uniform branch inside the loop (upper bound of the executed count)."""
import collections, os, re, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def compile_asm(out="/tmp/hk_kernels.s"):
    sys.path.insert(0, ROOT)
    from hpmpc_amd.build import ARCH, HIPCC, KFLAGS
    src = os.path.join(ROOT, "hpmpc_amd", "csrc", "hpmpc_kernels.hip")
    extra = os.environ.get("HK_COUNT_FLAGS", "").split()  # e.g. -DHK_COUNT_FIXED -DHK_COUNT_NOFALLBACK
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "--cuda-device-only", "-S"] + KFLAGS +
                   extra + [src, "-o", out], check=True, stderr=subprocess.DEVNULL)
    return out


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else compile_asm()
    kern = None
    loops = collections.OrderedDict()
    cur = None
    for ln in open(path):
        m = re.match(r"^(_Z\w*?(hk4?_[a-z_0-9]+)\w*|hk4?_\w+):", ln)
        if m:
            full = m.group(1)
            base = m.group(2) or full
            cls = "fix" + "x".join(re.findall(r"Li(\d+)E", full)) if "FixSh" in full else ("gen" if "NoFix" in full else "")
            kern = f"{base}<{cls}>" if cls else base
            continue
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):.*?(?:Loop Header: Depth=(\d)|Header=(BB\d+_\d+) Depth=(\d))?\s*$", ln)
        if ln.startswith(".LBB") or ln.startswith("; %bb."):
            cur = None
            hm = re.search(r"Inner Loop Header: Depth=(\d)", ln)
            if hm:
                lab = ln.split(":")[0].lstrip(".").replace("LBB", "BB")
                cur = (kern, lab)
            else:
                hm = re.search(r"Header=(BB\d+_\d+) Depth=(\d)", ln)
                if hm:
                    cur = (kern, hm.group(1))
            continue
        if cur and ln.startswith("\t") and not ln.strip().startswith((";", ".")):
            op = ln.split()[0]
            d = loops.setdefault(cur, collections.Counter())
            k = ("scratch" if op.startswith("scratch_") else "nop" if op == "s_nop" else "wait" if op.startswith("s_waitcnt") else "mfma" if "mfma" in op else "vmem" if op.startswith("buffer") or op.startswith("global") else
                 "lds" if op.startswith("ds_") else "salu" if op.startswith("s_") else
                 "lane" if ("readlane" in op or "writelane" in op or "readfirstlane" in op) else
                 "xlane" if ("dpp" in op or "permlane" in op) else "valu")
            d[k] += 1
            d["total"] += 1
    for (k, lab), d in loops.items():
        if d["total"] < 60:
            continue
        print(f"{k:26s} {lab:10s} total {d['total']:5d}  valu {d['valu']:4d} salu {d['salu']:4d} nop {d['nop']:3d} "
              f"wait {d['wait']:3d} lane {d['lane']:3d} xlane {d['xlane']:3d} vmem {d['vmem']:3d} lds {d['lds']:3d} "
              f"mfma {d['mfma']:2d} scratch {d['scratch']:3d}")


if __name__ == "__main__":
    main()
