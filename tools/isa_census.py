"""Static instruction census of one kernel, bucketed by source function and line.

python tools/isa_census.py SRC.hip KERNEL_REGEX [--lines N] [--fn FUNC_REGEX] [--range A:B]

Compiles SRC (device code only, the product's flags plus -gline-tables-only, so the code is the product's)
for gfx950, disassembles the code object with line info (llvm-objdump -d -l) and attributes every
instruction of the kernel(s) matching KERNEL_REGEX to the innermost source line the line table gives
(inlined device functions keep their own lines) and to the device function whose body holds that line.
Classes: f64 VALU (v_*_f64 arithmetic, compares and conversions), other VALU, 64-bit moves / selects
(v_mov_b64, v_cndmask pairs are counted as other VALU), SALU, SMEM, VMEM, LDS, branches / waits.
Static counts: an instruction in a loop counts once; the walker and path loops are where nearly all of
a megakernel's code is, so the shares are indicative of where its issue slots go, not a profile.
--range A:B restricts to the instructions of one source file's lines A..B; --prio N to the N-th (from 1) stretch
of code between an `s_setprio 1` and the next `s_setprio 0` in address order (the role-split pool's walker
loop: k_megakernel_roles_f64 has one per ancestor-column form)."""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950", "-munsafe-fp-atomics",
         "-gline-tables-only", "--cuda-device-only", "-c"]
# a function definition starts at column 0 (its body is indented): the last identifier before the first "("
# (or, inside a struct, at an indent of at most 4 with RT_DEV: a member function)
FN_DEF = re.compile(r"^(?:template\s*<[^>]*>\s*)?[A-Za-z_][\w:<>,*&\s]*?\b(\w+)\s*\(|^ {1,4}(?:static\s+)?RT_DEV\b[\w:<>,*&\s]*?\b(\w+)\s*\(")


def disasm(src, extra):
    tmp = tempfile.mkdtemp(prefix="isa_")
    co, elf = os.path.join(tmp, "k.co"), os.path.join(tmp, "k.elf")
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, src, "-o", co], check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={co}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={elf}"], check=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "-l", elf], check=True, capture_output=True,
                          text=True).stdout


_fn_cache = {}


def function_of(path, line):
    """The name of the function whose definition most closely precedes `line` in `path`."""
    if path not in _fn_cache:
        names = []
        try:
            with open(path) as f:
                lines = f.read().split("\n")
        except OSError:
            lines = []
        cur = "?"
        for i, text in enumerate(lines, 1):
            m = FN_DEF.match(text)
            name = (m.group(1) or m.group(2)) if m else None
            if m and name not in ("if", "for", "while", "switch", "return", "sizeof", "defined", "static_assert",
                                        "__attribute__", "typedef", "enum", "struct", "template"):
                cur = name
            names.append(cur)
        _fn_cache[path] = names
    names = _fn_cache[path]
    return names[line - 1] if 0 < line <= len(names) else "?"


def classify(op):
    if op.startswith(("s_waitcnt", "s_branch", "s_cbranch", "s_setprio", "s_barrier", "s_nop", "s_sleep",
                      "s_endpgm")):
        return "branch_wait"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_"):
        if re.search(r"_f64(_e32|_e64)?$", op) or op.startswith(("v_fma_f64", "v_div_", "v_rcp_f64", "v_rsq_f64",
                                                                  "v_sqrt_f64", "v_ldexp_f64", "v_frexp")):
            return "valu_f64"
        return "valu_other"
    return "other"


def main():
    args = [a for a in sys.argv[1:]]
    src, kre = args[0], re.compile(args[1])
    nlines = int(args[args.index("--lines") + 1]) if "--lines" in args else 40
    fnre = re.compile(args[args.index("--fn") + 1]) if "--fn" in args else None
    rng = None
    if "--range" in args:
        a, b = args[args.index("--range") + 1].split(":")
        rng = (int(a), int(b))
    prio = int(args[args.index("--prio") + 1]) if "--prio" in args else 0
    extra = args[args.index("--") + 1:] if "--" in args else []
    text = disasm(src, extra)
    by_fn = collections.defaultdict(collections.Counter)
    by_line = collections.defaultdict(collections.Counter)
    ops = collections.Counter()
    loc = ("?", 0)
    inside = False
    kernels = []
    nprio, in_prio = 0, False
    for ln in text.split("\n"):
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", ln)
        if m:
            inside = bool(kre.search(m.group(1)))
            if inside:
                kernels.append(m.group(1))
            continue
        if not inside:
            continue
        m = re.match(r"^; (/\S+):(\d+)", ln)
        if m:
            loc = (m.group(1), int(m.group(2)))
            continue
        m = re.match(r"^\t([a-z_0-9]+)", ln)
        if not m:
            continue
        op = m.group(1)
        if prio:
            if op == "s_setprio" and ln.split()[1] == "1" and not in_prio:
                nprio += 1
                in_prio = True
            elif op == "s_setprio" and ln.split()[1] == "0":
                in_prio = False
            if not (in_prio and nprio == prio):
                continue
        if rng and not (loc[1] >= rng[0] and loc[1] <= rng[1]):
            continue
        fn = function_of(loc[0], loc[1])
        if fnre and not fnre.search(fn):
            continue
        c = classify(op)
        key = f"{os.path.basename(loc[0])}:{fn}"
        by_fn[key][c] += 1
        by_line[f"{os.path.basename(loc[0])}:{loc[1]}"][c] += 1
        if c.startswith("valu"):
            ops[op] += 1
    print(f"kernels: {len(kernels)}: {kernels[:4]}{' ...' if len(kernels) > 4 else ''}")
    tot = collections.Counter()
    for v in by_fn.values():
        tot.update(v)
    print("total:", dict(tot))
    cls = ["valu_f64", "valu_other", "salu", "smem", "vmem", "lds", "branch_wait"]
    print(f"{'function':60s} " + " ".join(f"{c:>10s}" for c in cls))
    for k, v in sorted(by_fn.items(), key=lambda kv: -(kv[1]["valu_f64"] + kv[1]["valu_other"]))[:nlines]:
        print(f"{k[:60]:60s} " + " ".join(f"{v[c]:10d}" for c in cls))
    print("\ntop lines by VALU:")
    for k, v in sorted(by_line.items(), key=lambda kv: -(kv[1]["valu_f64"] + kv[1]["valu_other"]))[:nlines]:
        print(f"  {k:40s} f64 {v['valu_f64']:5d} other {v['valu_other']:5d} salu {v['salu']:5d}")
    print("\ntop VALU opcodes:")
    for op, n in ops.most_common(nlines):
        print(f"  {op:32s} {n}")


if __name__ == "__main__":
    main()
