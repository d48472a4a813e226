"""N-branch on-device gate (configs C4 / C5; VERDICT r03 missing #3): gm_gate_strong_step_n
behind the norms+SGD pass and the MMTM_N kernels gated from device memory reproduce the
host gate's N-branch rule (callbacks.bdr_decision: spread = max - min of the BDRs, caring =
argmax; reference rule src/callbacks.py:240-263 at N = 2) step by step: decisions, d_BDR,
losses, parameters and running averages; one captured graph serves every setting."""
import pytest
import torch

pytestmark = pytest.mark.gpu

V = 4


def _run(device_gate, graphs, steps, dev, V=V):
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN_N
    torch.manual_seed(0)
    m = MMTM_MVCNN_N(num_views=V, trunk="resnet18").to(dev)
    gate = Bias_Mitigation_Strong(epsilon=2e-3, curation_windowsize=2, branchnames=m.branch_names(),
                                  starting_epoch=1, MMTMnames=m.mmtm_names())
    st = BalancedStep(m, lr=0.05, gate=gate, graphs=graphs, device_gate=device_gate,
                      branchnames=m.branch_names(), MMTMnames=m.mmtm_names())
    assert st.device_gate == device_gate
    if device_gate:
        assert st.gate_n
    else:  # host flags through the same gated kernels: bitwise comparable
        for i in (2, 3, 4):
            getattr(m, f"mmtm{i}").mask_curation = True
    st.on_epoch_begin(1)
    g = torch.Generator(device=dev).manual_seed(5)
    xs = [torch.randn(4, V, 3, 64, 64, device=dev, generator=g) for _ in range(3)]
    ys = [torch.randint(0, 40, (4,), device=dev, generator=g) for _ in range(3)]
    trace = []
    for i in range(steps):
        loss = st(xs[i % 3], ys[i % 3])
        if device_gate:
            st.sync_gate()
        trace.append((float(loss), gate.d_BDR, st.flags.curation_mode, st.flags.caring_modality))
    return m, st, trace


@pytest.mark.parametrize("graphs,views", [(False, V), (True, V), (True, 2)])
def test_n_branch_device_gate_equals_host_gate(graphs, views):
    """At two views the N-branch kernel must log the reference's SIGNED d_BDR = BDR_0 - BDR_1
    (what the host gate's nb == 2 rule computes) and fill the two-branch host mirrors."""
    dev = torch.device("cuda:0")
    m_h, st_h, tr_h = _run(False, False, 10, dev, views)
    m_d, st_d, tr_d = _run(True, graphs, 10, dev, views)
    if views == 2:
        g_h, g_d = st_h.gate, st_d.gate
        for k in ("M_bypass_modal_0", "M_bypass_modal_1", "M_main_modal_0", "M_main_modal_1"):
            assert getattr(g_d, k) == pytest.approx(getattr(g_h, k), rel=1e-6), k
    assert {t[2] for t in tr_h} == {True, False}, "the trace should contain curation steps"
    assert len({t[3] for t in tr_h if t[2]}) >= 1
    if graphs:
        assert len(st_d._graphs) == 1
    diffs = [(a[0] - b[0], a[1] - b[1], a[2:], b[2:]) for a, b in zip(tr_h, tr_d)]
    for a, b in zip(tr_h, tr_d):
        assert a[2:] == b[2:], diffs
        assert a[0] == pytest.approx(b[0], rel=1e-6, abs=1e-6), diffs
        assert a[1] == pytest.approx(b[1], rel=1e-6, abs=1e-9), diffs
    sh, sd = m_h.state_dict(), m_d.state_dict()
    for k in sh:
        torch.testing.assert_close(sd[k], sh[k], rtol=1e-6, atol=1e-6, msg=k)
    for i in (2, 3, 4):
        a, b = getattr(m_h, f"mmtm{i}"), getattr(m_d, f"mmtm{i}")
        for ra, rb in zip(a.running_avg, b.running_avg):
            torch.testing.assert_close(rb, ra, rtol=1e-6, atol=1e-7)


def test_n_branch_gate_kernel_rule():
    """The decision kernel alone on hand-made group sums: BDR_i, spread, argmax (first on
    ties), the curation window and the locked (not unlocked) path."""
    import math
    from greedy_multimodal_learning_amd import _lib as L
    dev = torch.device("cuda:0")
    nb = 5
    st = L.GateStateN()
    st.nb, st.eps, st.window, st.unlock, st.caring = nb, 0.05, 2, 1, -1
    state = torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)
    # w, g per group: main0..4 then bypass0..4; BDR_i = log10((gb/wb) / (gm/wm))
    ratios = [(1.0, 2.0), (1.0, 1.0), (3.0, 3.0), (1.0, 2.0), (0.5, 4.0)]  # (main g/w, bypass g/w)
    s = []
    for rm, _ in ratios:
        s += [2.0, 2.0 * rm]
    for _, rb in ratios:
        s += [4.0, 4.0 * rb]
    sums = torch.tensor(s, dtype=torch.float64, device=dev)
    lib = L.load()

    def step():
        L.check(lib.gm_gate_strong_step_n(sums.data_ptr(), state.data_ptr(), L.stream_of(dev)), "gate_n")
        torch.cuda.synchronize()
        return L.GateStateN.from_buffer_copy(state.cpu().numpy().tobytes())

    r = step()
    bdr = [math.log10(rb / rm) for rm, rb in ratios]
    assert [round(v, 12) for v in r.bdr[:nb]] == [round(v, 12) for v in bdr]
    assert r.d_bdr == pytest.approx(max(bdr) - min(bdr), abs=1e-12)
    assert r.curation_mode == 1 and r.caring == 4 and r.curation_step == 0  # argmax: log10(8)
    r = step()
    assert r.curation_mode == 1 and r.curation_step == 1 and r.M_main[0] == pytest.approx(1.0)  # no update
    r = step()
    assert r.curation_mode == 0 and r.curation_step == 2 and r.n_curated == 2
    # ties: branches 0 and 3 share the max after making 4 equal to them -> first wins
    st2 = L.GateStateN.from_buffer_copy(bytes(st))
    state.copy_(torch.frombuffer(bytearray(bytes(st2)), dtype=torch.uint8))
    ratios[4] = (1.0, 2.0)
    s = []
    for rm, _ in ratios:
        s += [2.0, 2.0 * rm]
    for _, rb in ratios:
        s += [4.0, 4.0 * rb]
    sums.copy_(torch.tensor(s, dtype=torch.float64))
    r = step()
    assert r.curation_mode == 1 and r.caring == 0
    # locked: d computed, never curates
    st3 = L.GateStateN.from_buffer_copy(bytes(st))
    st3.unlock = 0
    state.copy_(torch.frombuffer(bytearray(bytes(st3)), dtype=torch.uint8))
    r = step()
    assert r.curation_mode == 0 and r.caring == 0 and r.d_bdr > 0.05
    # two branches: the signed d = BDR_0 - BDR_1 (negative when branch 1 leads), caring 1
    st4 = L.GateStateN()
    st4.nb, st4.eps, st4.window, st4.unlock, st4.caring = 2, 0.05, 2, 1, -1
    state.copy_(torch.frombuffer(bytearray(bytes(st4)), dtype=torch.uint8))
    sums2 = torch.tensor([2.0, 2.0, 2.0, 2.0, 4.0, 4.0, 4.0, 16.0], dtype=torch.float64, device=dev)
    L.check(lib.gm_gate_strong_step_n(sums2.data_ptr(), state.data_ptr(), L.stream_of(dev)), "gate_n")
    torch.cuda.synchronize()
    r = L.GateStateN.from_buffer_copy(state.cpu().numpy().tobytes())
    assert r.d_bdr == pytest.approx(-math.log10(4.0), abs=1e-12)
    assert r.curation_mode == 1 and r.caring == 1


@pytest.mark.parametrize("nb", [2, 5])
def test_group_sumsq_gate_matches_two_launches(nb):
    """gm_group_sumsq_gate (the gate's step rule run by the group-sum finalize's thread 0, no gate
    launch) == gm_group_sumsq followed by gm_gate_strong_step / _n: the same sums, the same
    updated parameters (fused SGD) and a bit-identical gate state, over several steps (the
    two-branch state for nb = 2 through the 4-group table, the N-branch state for nb = 5)."""
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd.callbacks import GroupNorms
    dev = torch.device("cuda:0")
    torch.manual_seed(nb)
    branches = [f"net_view_{i}" for i in range(nb)]
    mods = [f"mod{i}" for i in range(nb)]
    names = [f"net_view_{i}.conv{k}.weight" for i in range(nb) for k in range(3)] + \
            [f"mmtm{k}.fc_{m}.weight" for m in mods for k in range(2)]
    params = []
    for i, _ in enumerate(names):
        p = torch.randn(1000 + 37 * i, device=dev)
        params.append((p, torch.randn_like(p) * (0.1 + 0.05 * (i % 7))))
    lib = L.load()
    two = nb == 2

    def new_state():
        st = L.GateState() if two else L.GateStateN()
        if not two:
            st.nb = nb
        st.eps, st.window, st.unlock, st.caring = 1e-3, 2, 1, -1
        return torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)

    out = {}
    for fused in (True, False):
        ps = [torch.nn.Parameter(p.clone()) for p, _ in params]
        for q, (_, gr) in zip(ps, params):
            q.grad = gr.clone()
        norms = GroupNorms(list(zip(names, ps)), branches, mods)
        state = new_state()
        sums_seen = []
        for _ in range(4):
            if fused:
                s = norms.sums(lr=0.01, gate=state, gate_n=not two)
            else:
                s = norms.sums(lr=0.01)
                fn = lib.gm_gate_strong_step if two else lib.gm_gate_strong_step_n
                L.check(fn(s.data_ptr(), state.data_ptr(), L.stream_of(dev)), "gate")
            sums_seen.append(s.clone())
        torch.cuda.synchronize()
        out[fused] = (sums_seen, [p.detach().clone() for p in ps], state.cpu().clone())
    a, b = out[True], out[False]
    for x, y in zip(a[0], b[0]):
        assert torch.equal(x, y)
    for x, y in zip(a[1], b[1]):
        assert torch.equal(x, y)
    assert torch.equal(a[2], b[2]), "gate state differs"
