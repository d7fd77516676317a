"""ISA audit of the shipped code object (CPU test, no GPU needed).

The form-21 tableau pass (dlp_defer.hip, pass_d_kernel) issues v_fmac_f64_dpp
from inline asm, where the compiler's hazard recognizer cannot see it.  gfx9
requires two wait states between a VALU write of a VGPR and a DPP read of it;
the kernel is written so that the DPP source (a coefficient register) is only
ever written by a vector-memory load.  This test disassembles the gfx950 code
objects bundled in libdlp.so and checks, for every v_fmac_f64_dpp, that no VALU
instruction writing its DPP source sits within the two preceding wait states
(straight-line scan; the fused DPP instructions live in unrolled straight-line
code)."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "distributedlpsolver_amd", "libdlp.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _regs(tok):
    tok = tok.strip().lstrip("-")
    m = re.match(r"v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def _disasm():
    if not os.path.exists(SO) or not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("libdlp.so or llvm-objdump missing")
    d = tempfile.mkdtemp()
    try:
        shutil.copy(SO, os.path.join(d, "libdlp.so"))
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", "libdlp.so"], cwd=d,
                       check=True, capture_output=True)
        out = []
        for f in sorted(os.listdir(d)):
            if "amdgcn" in f and "gfx950" in f:
                r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", f], cwd=d,
                                   check=True, capture_output=True, text=True)
                out.append(r.stdout)
        return "\n".join(out)
    finally:
        shutil.rmtree(d, ignore_errors=True)


def test_fused_dpp_fma_has_no_valu_write_hazard():
    text = _disasm()
    instrs = []
    for line in text.splitlines():
        line = line.split("//")[0].strip()
        if not line or line.endswith(":") or line.startswith(("Disassembly", ";")) or "file format" in line:
            continue
        instrs.append(line)
    n_dpp = 0
    for i, ins in enumerate(instrs):
        op = ins.split()[0]
        if op != "v_fmac_f64_dpp":
            continue
        n_dpp += 1
        src0 = _regs(ins.split(None, 1)[1].split(",")[1])
        assert src0, ins
        waits = 0
        k = i - 1
        while k >= 0 and waits < 2:
            p = instrs[k]
            pop = p.split()[0]
            if pop.startswith("s_nop"):
                waits += int(p.split()[1], 0) + 1
                k -= 1
                continue
            if pop.startswith("v_") and not pop.startswith(("v_readlane", "v_readfirstlane", "v_cmp")):
                dst = _regs(p.split(None, 1)[1].split(",")[0]) if len(p.split()) > 1 else set()
                assert not (dst & src0), f"DPP hazard: '{p}' then '{ins}'"
            waits += 1
            k -= 1
    # the form-21 full-block instances (nt and plain): 64 steps x 2 rows x 2 unrolled groups
    assert n_dpp >= 512, n_dpp


def _readelf(d, f, *args):
    return subprocess.run([os.path.join(LLVM, "llvm-readelf"), *args, f], cwd=d, check=True,
                          capture_output=True, text=True).stdout


def _vgpr_counts():
    """{kernel symbol: VGPRs per lane} of the bundled code objects, as the hardware allocates them.

    Both the metadata note (.vgpr_count) and the kernel descriptor (<kernel>.kd: 64 bytes, the
    granulated count in compute_pgm_rsrc1 bits 5:0, granules of 8 VGPRs on gfx950) are read and
    the larger kept: hipcc can write a descriptor far above the note (a kernel with 64 KB of
    static LDS got 176 for a body of 30 VGPRs), and the descriptor is what the CU allocates."""
    if not os.path.exists(SO) or not os.path.exists(os.path.join(LLVM, "llvm-readelf")):
        pytest.skip("libdlp.so or llvm-readelf missing")
    d = tempfile.mkdtemp()
    try:
        shutil.copy(SO, os.path.join(d, "libdlp.so"))
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", "libdlp.so"], cwd=d,
                       check=True, capture_output=True)
        counts, name = {}, None
        for f in sorted(os.listdir(d)):
            if "amdgcn" in f and "gfx950" in f:
                for line in _readelf(d, f, "--notes").splitlines():
                    line = line.strip()
                    if line.startswith(".name:"):
                        name = line.split(":", 1)[1].strip()
                    elif line.startswith(".vgpr_count:") and name:
                        counts[name] = int(line.split(":", 1)[1])
                secs = []   # (addr, offset, size) of every section
                for line in _readelf(d, f, "-S", "--wide").splitlines():
                    m = re.match(r"\s*\[\s*\d+\]\s+\S+\s+\S+\s+([0-9a-f]+)\s+([0-9a-f]+)\s+([0-9a-f]+)", line)
                    if m:
                        secs.append(tuple(int(x, 16) for x in m.groups()))
                blob = open(os.path.join(d, f), "rb").read()
                for line in _readelf(d, f, "-s", "--wide").splitlines():
                    p = line.split()
                    if len(p) >= 8 and p[7].endswith(".kd"):
                        addr = int(p[1], 16)
                        off = next(o + addr - a for a, o, n in secs if a <= addr < a + n)
                        rsrc1 = int.from_bytes(blob[off + 48:off + 52], "little")
                        k = p[7][:-3]
                        counts[k] = max(counts.get(k, 0), ((rsrc1 & 63) + 1) * 8)
        return counts
    finally:
        shutil.rmtree(d, ignore_errors=True)


def test_lookahead_kernels_fit_beside_the_form21_pass():
    """Lookahead at K = 64 works only if the LEAN selection kernels share a CU with the
    form-21 pass: 3 pass waves x 160 VGPRs per SIMD leave 32 of the 512.
    A kernel that grows past those budgets silently serialises the chain behind the pass."""
    c = _vgpr_counts()
    def one(sub):
        hits = [v for k, v in c.items() if sub in k]
        assert hits, sub
        return max(hits)
    assert one("pass_d_kernel") <= 160, c
    assert one("pass_m_kernel") <= 160, c   # form 22 beside the chain (round 5: publishing)
    # its chain kernels: 3 form-22 waves (<= 136 allocated VGPRs each) leave 104 per SIMD
    assert one("ratio_mid_kernel") <= 104 and one("prow_mid_kernel") <= 104, c
    assert one("ratio_lean_kernel") <= 32   # every instance (ring depths 8 / 16, LCH 4 / 8)
    assert one("prow_lean_kernel") <= 32
    assert one("pivot_x_lean_kernel") <= 32   # the one-launch peer pivot beside the pass


def _functions(text):
    """{symbol: [instruction lines]} of the disassembly."""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line.strip())
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        line = line.split("//")[0].strip()
        if cur is not None and line and not line.endswith(":"):
            cur.append(line)
    return funcs


def test_peer_row_push_is_drained():
    """The peer exchange publishes the pivot row in the drained form (include/dlp.h, DESIGN.md
    §5): every lane's 16-B system-scope (sc0 sc1) store of its two row words, then
    s_waitcnt vmcnt(0) and a workgroup barrier, then the chunk flag (an 8-B sc0 sc1 store):
    no flag store may come before the wait and the barrier.  (The elements of the 16-B store
    are built from scalars: round 3's hipcc bit-cast of a vector element pushed the even
    column twice; the source guard below keeps that out.)"""
    funcs = _functions(_disasm())
    checked = 0
    for name, ins in funcs.items():
        if not any(k in name for k in ("prow_defer_kernel", "prow_lean_kernel", "xrow_send_kernel")):
            continue
        k = next((i for i, x in enumerate(ins) if x.startswith("buffer_store_dwordx4") and "sc0 sc1" in x), None)
        assert k is not None, name
        seen_wait = seen_bar = False
        for x in ins[k + 1:]:
            if x.startswith("s_waitcnt") and "vmcnt(0)" in x:
                seen_wait = True
            if x.startswith("s_barrier"):
                seen_bar = True
            if x.startswith(("global_store_dwordx2", "flat_store_dwordx2")) and "sc0 sc1" in x:
                assert seen_wait and seen_bar, (name, x)
                break
        else:
            raise AssertionError(f"{name}: no flag store after the row push")
        checked += 1
    assert checked >= 3, checked


def test_no_bit_cast_of_a_vector_element_in_kernels():
    """Source guard for the same compiler behaviour: no __builtin_bit_cast of a .x/.y/.z/.w
    element or a subscripted element of an ext_vector value in the kernel sources (round 5: a
    doubly subscripted operand, acc[t][i] of a d4 array, is caught too; dbits() is the form to use)."""
    pat = re.compile(r"__builtin_bit_cast\(\s*\w+\s*,\s*([\w\[\]]+\.[xyzw]|\w+\[[^\]]+\]\[[^\]]+\])\s*\)")
    csrc = os.path.join(ROOT, "distributedlpsolver_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h")):
            with open(os.path.join(csrc, f)) as fh:
                for k, line in enumerate(fh, 1):
                    code = line.split("//")[0]
                    assert not pat.search(code), f"{f}:{k}: {line.strip()}"


def test_band_publication_is_drained():
    """Band publication relies on the write-through hand-off form
    (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1 table) rather than
    release / acquire fences, which on gfx950 write back / invalidate the whole XCD L2 (ADVICE
    r03).  Pinned here on the shipped code object: the publishing passes store every output
    row write-through (sc1) and add to the band counter only behind s_waitcnt vmcnt(0) and a
    workgroup barrier; the LEAN selection kernels poll the counter with sc1 loads and read the
    published rows with sc1 loads."""
    funcs = _functions(_disasm())
    pubs = [n for n in funcs if ("pass_d_kernelILb1ELb1E" in n or
                                 (n.startswith("_ZN3dlp12_GLOBAL__N_113pass_q_kernel") and n.count("ELb1EE")) or
                                 ("pass_m_kernelILb1ELi2ELb1E" in n))]
    assert len(pubs) >= 3 and any("pass_m_kernel" in n for n in pubs), pubs
    for name in pubs:
        ins = funcs[name]
        stores = [x for x in ins if x.startswith("buffer_store")]
        assert stores and all(" sc1" in x for x in stores), (name, stores[:3])
        k = max(i for i, x in enumerate(ins) if x.startswith("global_atomic_add"))
        bar = max(i for i in range(k) if ins[i].startswith("s_barrier"))
        wait = max(i for i in range(bar) if ins[i].startswith("s_waitcnt") and "vmcnt(0)" in ins[i])
        assert not any(x.startswith(("buffer_store", "global_store")) for x in ins[wait:k]), name
    for sub in ("ratio_lean_kernelILi128ELi0E", "prow_lean_kernel"):
        ins = next(v for n, v in funcs.items() if sub in n)
        assert any(re.match(r"global_load_dword\b.*\bsc1\b", x) for x in ins), sub       # the counter
        assert any(re.match(r"global_load_dwordx2\b.*\bsc1\b", x) for x in ins), sub     # the rows
