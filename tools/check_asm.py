"""Static check of the gfx950 code objects in vit.rs_amd/build/*.o for LDS reads issued as inline asm.

The transposed LDS reads (ds_read_b64_tr_b16) are issued as inline asm (common.h
ds_read_tr16_asm): the compiler does not count them on lgkmcnt, so nothing but the kernel's own
`s_waitcnt lgkmcnt(..)` protects their destination registers.  A compiler-inserted copy (v_mov, a
shuffle, a spill) or any other instruction that touches such a register before a wait that retires
the read would use stale data.  This scans every kernel's disassembly in program order and reports

  * any instruction that mentions a destination VGPR of an asm transposed read that may still be
    outstanding on some path to it (data flow over the kernel's branches and loop back edges).

A read is retired by `s_waitcnt lgkmcnt(N)` once at least N younger LDS instructions (ds_*) were
issued after it (LDS operations complete in order), or by lgkmcnt(0).

Second rule (engine bit-identity): the x-aux epilogue with column sums
(EPI_BF16_MUL = 9, the fcproj dgrad) must round its products before summing them in every GEMM
engine, so no kernel instantiated for it may contain a float FMA (gemm_common.h pins
`#pragma clang fp contract(off)` there; hipcc contracted `v *= aux; cs += v` in some engines and
not in others, and their column sums then differed in the last bits).

    python tools/check_asm.py [objects...]        exit status 1 on a violation
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")


def regs_of(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def disassemble(obj, tmp):
    fb = os.path.join(tmp, "fb.bin")
    co = os.path.join(tmp, "co.o")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", obj], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--targets={TARGET}", f"--input={fb}",
                    f"--output={co}", "--unbundle"], check=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                          capture_output=True, text=True).stdout


def parse(dis):
    """-> {kernel: [(addr, op, operands)]} in address order"""
    funcs, fn = {}, None
    for raw in dis.splitlines():
        m = FUNC.match(raw.strip())
        if m:
            fn = m.group(1)
            funcs[fn] = []
            continue
        if fn is None or "//" not in raw:
            continue
        code, comment = raw.split("//", 1)
        code = code.strip()
        am = re.match(r"\s*([0-9A-Fa-f]+):", comment)
        if not code or not am:
            continue
        op = code.split()[0]
        funcs[fn].append((int(am.group(1), 16), op, code[len(op):]))
    return funcs


def check_kernel(fn, ins):
    """Data flow over the kernel's control-flow graph.  State at an instruction: the set of
    outstanding asm transposed reads (read index, younger LDS ops since it, capped)."""
    index = {a: i for i, (a, _, _) in enumerate(ins)}
    reads = {}  # instruction index -> destination registers
    for i, (_, op, rest) in enumerate(ins):
        if op == "ds_read_b64_tr_b16":
            reads[i] = regs_of(rest.split(",")[0])
    if not reads:
        return False, []

    def succ(i):
        a, op, rest = ins[i]
        nxt = [i + 1] if i + 1 < len(ins) else []
        if op == "s_endpgm" or op.startswith("s_setpc"):
            return []
        if op == "s_branch" or op.startswith("s_cbranch"):
            imm = int(rest.split()[0])
            imm = imm - 65536 if imm >= 32768 else imm
            t = index.get(a + 4 + 4 * imm)
            tgt = [t] if t is not None else []
            return tgt if op == "s_branch" else tgt + nxt
        return nxt

    state = {0: frozenset()}
    work = [0]
    bad = {}
    while work:
        i = work.pop()
        cur = state[i]
        _, op, rest = ins[i]
        out = set(cur)
        if op == "s_waitcnt":
            lg = re.search(r"lgkmcnt\((\d+)\)", rest)
            if lg:
                n = int(lg.group(1))
                out = {p for p in out if p[1] < n} if n else set()
        else:
            if out:
                live = set().union(*[reads[r] for r, _ in out])
                # another transposed read may overwrite a pending destination (LDS returns in
                # order); its address operand must not be pending
                hit = regs_of(rest.split(",", 1)[1] if op == "ds_read_b64_tr_b16" else rest) & live
                if hit:
                    bad[i] = f"'{op}{rest}' touches v{sorted(hit)} before the wait retiring its asm read"
            if op.startswith("ds_"):
                out = {(r, min(c + 1, 64)) for r, c in out}
            if i in reads:
                out.add((i, 0))
        out = frozenset(out)
        for j in succ(i):
            old = state.get(j)
            new = out if old is None else old | out
            if new != old:
                state[j] = new
                work.append(j)
    return True, [(fn, bad[i]) for i in sorted(bad)]


def check_text(dis):
    """-> (kernels with asm transposed reads, violations)"""
    kernels, violations = set(), []
    for fn, ins in parse(dis).items():
        has, v = check_kernel(fn, ins)
        if has:
            kernels.add(fn)
        violations += v
    return kernels, violations


FMA_OP = re.compile(r"v_(pk_)?fmac?_f32|v_fma_mix|v_mad_f32|v_mac_f32|v_fma_f16")
EPI_MUL = re.compile(r"(I|E)Li9E")  # template argument EPI = 9 in the mangled kernel name


def colsum_fma_violations(dis):
    """-> [(kernel, count)] of EPI 9 GEMM kernels that contain float FMAs"""
    out = []
    for fn, ins in parse(dis).items():
        if "gemm" in fn and EPI_MUL.search(fn):
            n = sum(1 for _, op, _ in ins if FMA_OP.match(op))
            if n:
                out.append((fn, n))
    return out


def main(objs):
    objs = objs or sorted(glob.glob(os.path.join(ROOT, "vit.rs_amd", "build", "*.o")))
    total_k, total_v = 0, []
    with tempfile.TemporaryDirectory() as tmp:
        for o in objs:
            try:
                dis = disassemble(o, tmp)
            except subprocess.CalledProcessError:
                continue  # host-only object (no device code)
            k, v = check_text(dis)
            total_k += len(k)
            total_v += [(os.path.basename(o),) + x for x in v]
            total_v += [(os.path.basename(o), fn, f"{n} float FMA(s) in an EPI 9 (x aux + column sums) kernel")
                        for fn, n in colsum_fma_violations(dis)]
    for o, fn, msg in total_v[:50]:
        print(f"{o}: {fn}: {msg}")
    print(f"{total_k} kernels with asm transposed LDS reads checked, {len(total_v)} violation(s)")
    return 1 if total_v else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
