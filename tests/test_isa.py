"""Build-artefact checks on the gfx950 code objects of libadipose_hip.so (CPU only: the objects are disassembled,
nothing runs on a GPU).

* No kernel spills VGPRs to scratch except a committed list of opt-in / A-B instances. A spill in a hot kernel costs
  2-4x (round 5: an epilogue change made the halo weight gradient spill 134 VGPRs and run 3.5x slower), and the
  build gives no error for it.
* The persistent forward's in-loop tile claim (conv_common.h claim_issue / claim_publish, option tap64p_claim /
  dp_claim) keeps the returning atomic's destination VGPR in flight across the K loop; the hardware does not
  interlock a VGPR against a pending vector-memory return, so nothing may read or overwrite that register until a
  `s_waitcnt vmcnt(N)` that retires the atomic (N <= the vector-memory instructions issued after it). The check walks
  every control-flow path from each such atomic up to its publishing LDS store (round-4 ADVICE: the compiler could
  copy, spill or reuse the register in between, and a stale tile id would compute one tile twice and skip another).
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "adipose_tissue-unet_amd", "csrc", "build")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

# known spilling instances: opt-in variants (the 4-wave w4 forward, the 9-wave and claimed halo weight gradients,
# the claimed / BN-backward-reduction halo forwards, the tap64 kernel's mid-step-barrier and 128-wide forms) and one
# f32 helper; none is on the default bf16 training path
SPILL_OK = [
    r"igemm_fwd_w4_kernel<",
    r"igemm_fwd_halop_kernel<true, 1, 64, false, 0, false, true, false>",
    r"igemm_fwd_tap64_kernel<2, 4, 128, (true|false), false, false, (true|false), (-1|0|1|2)>",
    r"igemm_wgrad_halop_kernel<8, true, 8, true, false>",
    r"igemm_wgrad_halop_kernel<8, true, 4, true, false>",
    r"igemm_wgrad_halop_kernel<9, false, 8, true, false>",
    r"igemm_wgrad_halop_kernel<8, false, 8, true, false>",
    r"bn_bwd_apply_head_kernel<float, 4>",
]


def _tools_ok():
    return os.path.isdir(BUILD) and os.path.exists(os.path.join(LLVM, "clang-offload-bundler")) and shutil.which(
        "objcopy") is not None


pytestmark = pytest.mark.skipif(not _tools_ok(), reason="no build directory or ROCm LLVM tools")


def _code_object(obj, tmp):
    """The gfx950 code object of a hipcc-built host object (its .hip_fatbin offload bundle)."""
    fat = os.path.join(tmp, os.path.basename(obj) + ".fat")
    co = os.path.join(tmp, os.path.basename(obj) + ".co")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", f"--targets={TARGET}", f"--input={fat}",
                    f"--output={co}", "--unbundle"], check=True)
    return co


def _demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    return [o[o.find("::") + 2:] if "::" in o else o for o in out]


@pytest.fixture(scope="module")
def code_objects():
    objs = sorted(os.path.join(BUILD, f) for f in os.listdir(BUILD) if f.endswith(".hip.o"))
    tmp = tempfile.mkdtemp()
    try:
        yield {os.path.basename(o): _code_object(o, tmp) for o in objs}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def test_no_unexpected_vgpr_spills(code_objects):
    bad = []
    for name, co in code_objects.items():
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True,
                               text=True).stdout
        kn = re.findall(r"\.name:\s+(\S+)", notes)
        sp = [int(v) for v in re.findall(r"\.vgpr_spill_count:\s+(\d+)", notes)]
        assert len(kn) == len(sp), name
        for k, s in zip(_demangle(kn), sp):
            if s > 0 and not any(re.search(p, k) for p in SPILL_OK):
                bad.append((name, k, s))
    assert not bad, bad


_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def _regs(text):
    out = set()
    for m in _VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _disasm(co):
    """[(address, mnemonic, operand text)] of every instruction, in address order, per function."""
    text = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], capture_output=True, text=True).stdout
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
        if m and cur is not None:
            cur.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return funcs


def _is_vmem(op):
    return op.startswith(("buffer_", "global_", "flat_")) and op != "buffer_inv"


def _paths_ok(ins, start):
    """From the returning atomic at index `start`: on every control-flow path (conditions ignored), its destination
    register is neither read nor written -- no copy, spill, phi move or reuse -- before either the publishing
    `ds_write_b32 <ring>, vD` of claim_publish or an s_waitcnt vmcnt(N) with N <= (vector-memory instructions issued
    after the atomic on that path)."""
    addr_idx = {a: i for i, (a, _, _) in enumerate(ins)}
    dst = min(_regs(ins[start][2].split(",")[0]))
    stack = [(start + 1, 0)]
    seen = set()
    problems = []
    while stack:
        i, young = stack.pop()
        while i < len(ins):
            if (i, young) in seen:
                break
            seen.add((i, young))
            addr, op, opnd = ins[i]
            if op == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", opnd)
                if m and int(m.group(1)) <= young:
                    break   # retired on this path
            elif op == "s_endpgm":
                break
            elif op == "ds_write_b32" and _regs(opnd.split(",")[1]) == {dst} and dst not in _regs(opnd.split(",")[0]):
                break   # claim_publish: its own wait (or the caller's) sits in front of this store by construction
            elif dst in _regs(opnd):
                problems.append((hex(addr), op, opnd))
                break
            if _is_vmem(op):
                young += 1
            if op == "s_branch" or op.startswith("s_cbranch"):
                tgt = addr + 4 + 4 * int(opnd.split()[0])
                if tgt in addr_idx:
                    stack.append((addr_idx[tgt], young))
                if op == "s_branch":
                    break
            i += 1
    return problems


def test_claim_atomic_result_retired_before_use(code_objects):
    co = code_objects.get("conv_fwd_tap64p.hip.o")
    assert co is not None
    checked = 0
    bad = []
    for fn, ins in _disasm(co).items():
        for i, (addr, op, opnd) in enumerate(ins):
            # every returning (sc0) integer add: the claims (claim_issue in the loop, claim_next2 in the prologue)
            if op == "global_atomic_add" and opnd.endswith("sc0"):
                checked += 1
                p = _paths_ok(ins, i)
                if p:
                    bad.append((_demangle([fn])[0], hex(addr), p[:3]))
    assert checked > 0, "no claim atomic found in the persistent forward's code object"
    assert not bad, bad


def test_reported_kernel_names_exist(code_objects):
    """Every name the library reports for a launch (adp::set_kernel, read back by adp_last_kernel and used as the bench's
    roofline key) is the full demangled name of a kernel in the code objects, as rocprofv3 prints it: the per-kernel
    timing and the committed kernel-trace summaries must name the same instantiation (round 5: several names had
    dropped defaulted template arguments)."""
    src_dir = os.path.join(ROOT, "adipose_tissue-unet_amd", "csrc")
    pats = []
    for f in sorted(os.listdir(src_dir)):
        if f.endswith((".hip", ".cpp", ".h")):
            text = open(os.path.join(src_dir, f)).read()
            for m in re.finditer(r'set_kernel\(\s*"([A-Za-z0-9_]+_kernel<[^"]*>)"', text):
                pats.append((f, m.group(1)))
    assert len(pats) > 20
    names = set()
    for co in code_objects.values():
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True,
                               text=True).stdout
        for d in _demangle(re.findall(r"\.name:\s+(\S+)", notes)):
            names.add(d.split("(")[0])
    missing = []
    for f, p in pats:
        rx = re.escape(p).replace("%d", r"-?\d+").replace("%s", "(true|false)")
        if not any(re.fullmatch(rx, n) for n in names):
            missing.append((f, p))
    assert not missing, missing


def _ds_paths_ok(ins, start):
    """From an LDS read at index `start` (the kernels' fragment reads are inline asm, which hipcc does not count): on every
    control-flow path, its destination registers are neither read nor written -- no copy, spill or reuse -- before an
    s_waitcnt lgkmcnt(N) with N <= the LDS instructions issued after the read on that path (LDS operations return in
    order; scalar loads also count in lgkmcnt but only make such a wait stricter)."""
    addr_idx = {a: i for i, (a, _, _) in enumerate(ins)}
    dst = _regs(ins[start][2].split(",")[0])
    stack = [(start + 1, 0)]
    seen = set()
    while stack:
        i, young = stack.pop()
        while i < len(ins):
            if (i, young) in seen:
                break
            seen.add((i, young))
            addr, op, opnd = ins[i]
            if op == "s_waitcnt":
                m = re.search(r"lgkmcnt\((\d+)\)", opnd)
                if (m and int(m.group(1)) <= young) or opnd.strip() == "0":
                    break
            elif op == "s_endpgm":
                break
            elif dst & _regs(opnd):
                return [(hex(addr), op, opnd)]
            if op.startswith("ds_"):
                young += 1
            if op == "s_branch" or op.startswith("s_cbranch"):
                tgt = addr + 4 + 4 * int(opnd.split()[0])
                if tgt in addr_idx:
                    stack.append((addr_idx[tgt], young))
                if op == "s_branch":
                    break
            i += 1
    return []


@pytest.mark.parametrize("obj", ["conv_wgrad_tap64.hip.o", "conv_fwd_halo.hip.o", "conv_fwd_tap64p.hip.o",
                                 "conv_fwd_tap64.hip.o"])
def test_asm_lds_reads_untouched_until_waited(code_objects, obj):
    """The hot K loops read their MFMA fragments with inline-asm ds_read_b64_tr_b16 / ds_read_b128 (the builtins would make
    hipcc drain every LDS-DMA in flight first). hipcc treats an asm load's destination as written at the statement, so
    under register pressure it may copy or spill the register before the data lands (round 6: the first build of the
    tap-pair weight gradient spilled and moved fragment registers right after their reads; silent garbage, no fault).
    Every LDS read's destination must stay untouched until a wait that retires it."""
    co = code_objects.get(obj)
    assert co is not None
    bad = []
    n = 0
    for fn, ins in _disasm(co).items():
        for i, (addr, op, opnd) in enumerate(ins):
            if op.startswith("ds_read"):
                n += 1
                p = _ds_paths_ok(ins, i)
                if p:
                    bad.append((_demangle([fn])[0][:80], hex(addr), op, opnd, p[0]))
    assert n > 0
    assert not bad, bad[:5]


def test_pair_wgrad_mfma_operands_come_from_lds():
    """The tap-pair weight gradient's MFMAs are inline asm (accumulating in place), so hipcc pads no hazard in front of
    them: every A / B operand register must have been written last by one of the kernel's LDS reads (never by a VALU
    copy, which would need wait states before an MFMA reads it), and every accumulator is used in place (D = C)."""
    co = None
    for f in os.listdir(BUILD):
        if f == "conv_wgrad_tap64.hip.o":
            tmp = tempfile.mkdtemp()
            co = _code_object(os.path.join(BUILD, f), tmp)
    assert co is not None
    checked = 0
    bad = []
    for fn, ins in _disasm(co).items():
        if "halopair" not in fn:
            continue
        for i, (addr, op, opnd) in enumerate(ins):
            if not op.startswith("v_mfma"):
                continue
            parts = [p.strip() for p in opnd.split(",")]
            if parts[0] != parts[3]:
                bad.append((hex(addr), "D != C", opnd))
            for src in (parts[1], parts[2]):
                regs = _regs(src)
                j = i - 1
                while j >= 0:
                    _, op2, opnd2 = ins[j]
                    if op2.startswith("v_mfma") or op2.startswith("s_") or not opnd2:
                        j -= 1
                        continue
                    d = _regs(opnd2.split(",")[0])
                    if d & regs:
                        if not op2.startswith("ds_read"):
                            bad.append((hex(addr), op2, opnd2))
                        break
                    j -= 1
            checked += 1
    assert checked >= 144
    assert not bad, bad[:5]
