"""GPU parity of every phase-2 form of the batched placement path
(KSG_BATCH_MODE): "spec" (the default: the speculate-and-verify
walk in the two-stream pipeline, serialised with timing on), "window" (the
slot walk inside the pipeline with the two-batch window: the spec walk's
fallback outside its scope; also without the window and with per-kernel timing
on, which runs the same arithmetic without overlap) and "slot" (one launch
chain per batch, at 64- and 128-pod batches: the captured queues' form).
Same bar as the default path: placements, per-pod results and node state
bit-exact against the C++ oracle, including split calls.  (Round 6 retired
"scan", "topset" and "tcol".)"""
import numpy as np
import pytest

from conftest import pkg
from test_gpu_parity import CASES, _engine_with_batch_mode

G = pkg("generator")
E = pkg("encoder")


def _have_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not _have_gpu(), reason="needs an MI355X")]

# (mode, extra env).  "spec" is the default; "window" its fallback (the slot
# walk, one lane per slot, at 64-pod batches).
MODES = {"window": ("window", {}), "window-timed": ("window", {"_timing": 1}),
         "window-nowindow": ("window", {"KSG_PIPE_WINDOW": 0}), "slot": ("slot", {}),
         "slot128": ("slot", {"KSG_SLOT_BLOCK": 128}),
         "spec": ("spec", {}), "spec-timed": ("spec", {"_timing": 1})}


@pytest.fixture(scope="module", params=list(MODES))
def variant(request, built):
    mode, env = MODES[request.param]
    env = dict(env)
    timing = env.pop("_timing", 0)
    eng = _engine_with_batch_mode(mode, **env)
    if timing:
        eng.set_timing(True)
    return eng


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(8)


def _check(gpu, oracle, nodes, pods, prof, split=True):
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu.load(enc, pf)
    oracle.load(enc, pf)
    pg, rg = gpu.run_queue(0, len(pods))
    po, ro = oracle.run_queue(0, len(pods))
    np.testing.assert_array_equal(pg, po)
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)
    R = len(enc.cluster.res_names)
    for a, b in zip(gpu.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(a, b)
    if split:
        gpu.reset_state()
        half = len(pods) // 2
        p1, _ = gpu.run_queue(0, half)
        p2, _ = gpu.run_queue(half, len(pods) - half)
        np.testing.assert_array_equal(np.concatenate([p1, p2]), po)


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_variant_placements_match_oracle(variant, oracle, name, make):
    _check(variant, oracle, *make())


def test_variant_full_config2(variant, oracle):
    _check(variant, oracle, *G.config2(), split=False)


# ---- the 32-bit slot walk (KSG_RUN_SLOT32) ------------------------------------
native = pkg("native")


def test_slot32_runs_and_matches_int64(oracle):
    """Config 2 takes the 32-bit Fit / BalancedAllocation instances (memory in
    MiB, range-checked); the int64 instances (KSG_FORCE_PATH=3) and the oracle
    agree with it bit for bit."""
    nodes, pods, prof = G.config2(n_nodes=2000, n_pods=3000, seed=9)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    a = _engine_with_batch_mode("slot")
    b = _engine_with_batch_mode("slot", KSG_FORCE_PATH=3)
    out = []
    for eng in (a, b, oracle):
        eng.load(enc, pf)
        out.append(eng.run_queue(0, len(pods)))
    assert a.last_run_info() == (2, native.RUN_SLOT32)
    assert b.last_run_info() == (2, 0)
    for pl, res in out[1:]:
        np.testing.assert_array_equal(out[0][0], pl)
        for f in ("n_feasible", "status", "score_skip"):
            np.testing.assert_array_equal(out[0][1][f], res[f], err_msg=f)


def test_slot32_refused_on_sub_mib_memory(oracle):
    nodes, pods, prof = G.config2(n_nodes=300, n_pods=400, seed=9)
    nodes[3].allocatable["memory"] += 4096
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    a = _engine_with_batch_mode("slot")
    a.load(enc, pf)
    oracle.load(enc, pf)
    pl, _ = a.run_queue(0, len(pods))
    path, flags = a.last_run_info()
    assert path == 2 and not flags & native.RUN_SLOT32   # the int64 slot walk
    np.testing.assert_array_equal(pl, oracle.run_queue(0, len(pods))[0])


# ---- the speculate-and-verify walk (KSG_RUN_SPEC) ---------------------------------
@pytest.mark.parametrize("strategy,seed", [("least", 21), ("most", 21), ("least", 5)])
def test_spec_runs_and_matches_oracle(oracle, strategy, seed):
    """Config 2 runs phase 2 as the speculate-and-verify walk (ksched_phase2v.h).
    LeastAllocated mostly speculates right; MostAllocated re-chooses the node
    it packs, so nearly every pod is a mis-speculation corrected in its own
    round: both exercise the rollback, the re-choice versions and the pointer
    snapshots."""
    P = pkg("profile")
    nodes, pods, prof = G.config2(n_nodes=1500, n_pods=2500, seed=seed)
    if strategy == "most":
        prof = P.config2_profile(strategy=P.MOST_ALLOCATED)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    a = _engine_with_batch_mode("spec")
    a.load(enc, pf)
    oracle.load(enc, pf)
    pl, res = a.run_queue(0, len(pods))
    assert a.last_run_info() == (2, native.RUN_SLOT32 | native.RUN_SPEC)
    po, ro = oracle.run_queue(0, len(pods))
    np.testing.assert_array_equal(pl, po)
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(res[f], ro[f], err_msg=f)
    R = len(enc.cluster.res_names)
    for x, y in zip(a.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("overlap", [1, 0])
def test_spec_walk_guard_reaches_the_host(overlap):
    """The walk's broken-invariant word (a node index outside the cluster,
    or a round that committed nothing) is armed in every mode, the PMC passes'
    KSG_PIPE_OVERLAP=0 included: an injected report fails the call loudly."""
    nodes, pods, prof = G.config2(n_nodes=600, n_pods=400, seed=3)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    a = _engine_with_batch_mode("spec", KSG_PIPE_OVERLAP=overlap, KSG_TEST_INJECT_WALK_ERR=1)
    a.load(enc, pf)
    with pytest.raises(native.KschedError, match="invariant broken"):
        a.run_queue(0, len(pods))


# ---- the wide-memory instance of the spec walk (KSG_RUN_WIDE_MEM) ----------------
@pytest.mark.parametrize("strategy,n_nodes,n_pods", [("least", 1500, 2500), ("most", 1500, 2500),
                                                     ("least", 5000, 50000)])
def test_spec_wide_memory_matches_oracle(oracle, strategy, n_nodes, n_pods):
    """Kubelet-style memory (allocatable a whole number of Ki, not of Mi;
    decimal pod requests): outside the N32 forms, so the spec walk runs its
    wide-memory instance (memory in int64 bytes) and stays bit-exact."""
    P = pkg("profile")
    nodes, pods, prof = G.config2_kubelet(n_nodes=n_nodes, n_pods=n_pods)
    if strategy == "most":
        prof = P.config2_profile(strategy=P.MOST_ALLOCATED)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    a = _engine_with_batch_mode("spec")
    a.load(enc, pf)
    oracle.load(enc, pf)
    pl, res = a.run_queue(0, len(pods))
    assert a.last_run_info() == (2, native.RUN_SPEC | native.RUN_WIDE_MEM)
    po, ro = oracle.run_queue(0, len(pods))
    np.testing.assert_array_equal(pl, po)
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(res[f], ro[f], err_msg=f)
    R = len(enc.cluster.res_names)
    for x, y in zip(a.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(x, y)
