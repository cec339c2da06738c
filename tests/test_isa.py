"""The fused K0 + K1's grid barrier, pinned in the shipped ISA (VERDICT r04
item 3).  The barrier's correctness rests on gfx950's
memory pipeline, not on the HSA model's scopes alone: the handed-over data
(the zero words, each block's partial centroid box, the last block's
global box) is stored write-through (agent-scope atomic stores = `sc1`),
every wave drains its stores (`s_waitcnt vmcnt(0)`) before the block's
`s_barrier`, and only then does thread 0 arrive on (or open) the counter;
readers use agent-scope loads (`sc1`).  A compiler change that dropped the
drain or demoted a store would break the barrier silently -- this test
disassembles `k_morton_tb<true, 512>` from librtamd.so (CPU only: the
llvm-objdump of the image) and fails on it.  The kernel is
gpu_raytracer_amd/csrc/build_kernels.hip (grid_arrive_last / grid_open /
grid_wait and the FUSED branch of k_morton_tb)."""
import os
import re
import shutil
import subprocess

import pytest

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
LIB = os.path.join(os.path.dirname(__file__), "..", "gpu_raytracer_amd", "lib", "librtamd.so")
FUSED = "_ZN2rt11k_morton_tbILb1ELi512E"


@pytest.fixture(scope="module")
def fused_isa(tmp_path_factory):
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    assert os.path.exists(LIB), "build librtamd.so first (__graft_entry__.build())"
    d = tmp_path_factory.mktemp("isa")
    lib = d / "librtamd.so"
    shutil.copy(LIB, lib)  # --offloading writes the bundles beside its input
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, capture_output=True)
    objs = sorted(p for p in d.iterdir() if p.name.endswith("gfx950"))
    assert objs, "no gfx950 code object in librtamd.so"
    for o in objs:
        text = subprocess.run([OBJDUMP, "-d", str(o)], check=True, capture_output=True, text=True).stdout
        m = re.search(r"^[0-9a-f]+ <(" + FUSED + r"[^>]*)>:\n", text, re.M)
        if not m:
            continue
        body = text[m.end():]
        end = re.search(r"^[0-9a-f]+ <", body, re.M)
        body = body[: end.start()] if end else body
        ins = []
        for line in body.splitlines():
            t = line.split("//")[0].strip()
            if t:
                ins.append(t)
        return ins
    pytest.fail("k_morton_tb<true, 512> not found in librtamd.so")


def _op(i):
    return i.split()[0]


def _is_store(i):
    return _op(i).startswith(("global_store", "buffer_store", "flat_store"))


def _drains_vm(i):
    return _op(i) == "s_waitcnt" and "vmcnt(0)" in i


def _barrier_atomics(ins):
    at = [k for k, i in enumerate(ins) if _op(i) == "global_atomic_add"]
    assert len(at) >= 2, "expected the arrival and the opening RMW"
    return at[0], at[1]


def test_fused_barrier_stores_are_write_through(fused_isa):
    arrive, _ = _barrier_atomics(fused_isa)
    pre = [i for i in fused_isa[:arrive] if _is_store(i)]
    assert len(pre) >= 2, pre  # the zero words and the partial box
    for i in pre:
        assert re.search(r"\bsc1\b", i), "a pre-barrier store is not agent-scope write-through: " + i


@pytest.mark.parametrize("which", ["arrival", "open"])
def test_fused_barrier_drains_before_rmw(fused_isa, which):
    k = _barrier_atomics(fused_isa)[0 if which == "arrival" else 1]
    # walk back from the RMW: an s_barrier, and before it a vmcnt(0) drain,
    # must sit between the RMW and the nearest preceding store
    seen_barrier = drained = False
    store = None
    for i in reversed(fused_isa[:k]):
        if _is_store(i):
            store = i
            break
        if _op(i) == "s_barrier":
            seen_barrier = True
        elif seen_barrier and _drains_vm(i):
            drained = True
    assert store is not None
    assert re.search(r"\bsc1\b", store), "the published store is not write-through: " + store
    assert seen_barrier and drained, f"{which}: no s_waitcnt vmcnt(0) + s_barrier between '{store}' and the RMW"


def test_fused_barrier_reads_are_agent_scope(fused_isa):
    arrive, open_ = _barrier_atomics(fused_isa)
    ld = re.compile(r"^global_load_dword\b")
    # the poll loop: an sc1 load of the counter next to s_memrealtime
    poll = [i for i in fused_isa[arrive:open_] if ld.match(i)]
    assert any(re.search(r"\bsc1\b", i) for i in poll), poll
    assert any(_op(i) == "s_memrealtime" for i in fused_isa[arrive:open_])
    # every load between the arrival and the open (poll + the last block's
    # partial-box reduction) is agent-scope
    for i in poll:
        assert re.search(r"\bsc1\b", i), i
    # the global box, after the barrier: the first load after the open
    after = [i for i in fused_isa[open_:] if ld.match(i)]
    assert after and re.search(r"\bsc1\b", after[0]), after[:1]
