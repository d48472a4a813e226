"""Whole-step hipGraph capture (BalancedStep(graphs=True)) == eager steps: same
losses, gate decisions, parameters and every piece of device state (BN running
statistics and counters, MMTM running averages and step), across curation
switches (one graph per curation setting)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(graphs, steps, dev, bind=False):
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    torch.manual_seed(0)
    m = MMTM_MVCNN().to(dev)
    gate = Bias_Mitigation_Strong(epsilon=2e-3, curation_windowsize=2, branchnames=["net_view_0", "net_view_1"],
                                  starting_epoch=1)
    st = BalancedStep(m, lr=0.05, gate=gate, graphs=graphs, device_gate=False)
    st.on_epoch_begin(1)
    g = torch.Generator(device=dev).manual_seed(5)
    xs = [torch.randn(4, 2, 3, 64, 64, device=dev, generator=g) for _ in range(3)]
    ys = [torch.randint(0, 40, (4,), device=dev, generator=g) for _ in range(3)]
    if bind:
        st.bind_batches(*zip(xs, ys))
    trace = []
    for i in range(steps):
        loss = st(xs[i % 3], ys[i % 3])
        trace.append((float(loss), gate.d_BDR, st.flags.curation_mode, st.flags.caring_modality))
    return m, st, trace


def test_bound_batches_equal_copied_batches():
    """Batches bound as graph input slots (no copy, one graph per slot and setting)
    step exactly like batches copied into the engine's static buffers."""
    dev = torch.device("cuda:0")
    m_c, st_c, tr_c = _run(True, 7, dev)
    m_b, st_b, tr_b = _run(True, 7, dev, bind=True)
    assert len(st_b._graphs) > len(st_c._graphs)
    assert tr_b == tr_c
    sc, sb = m_c.state_dict(), m_b.state_dict()
    for k in sc:
        assert torch.equal(sb[k], sc[k]), k


def test_graph_steps_equal_eager_steps():
    dev = torch.device("cuda:0")
    m_e, st_e, tr_e = _run(False, 9, dev)
    m_g, st_g, tr_g = _run(True, 9, dev)
    assert len(st_g._graphs) >= 2, "curation switches should have produced several graphs"
    assert {t[2] for t in tr_e} == {True, False}
    for a, b in zip(tr_e, tr_g):
        assert a[2:] == b[2:]
        assert a[0] == pytest.approx(b[0], rel=1e-6, abs=1e-6)
        assert a[1] == pytest.approx(b[1], rel=1e-6, abs=1e-9)
    se, sg = m_e.state_dict(), m_g.state_dict()
    for k in se:
        torch.testing.assert_close(sg[k], se[k], rtol=1e-6, atol=1e-6, msg=k)
    for i in (2, 3, 4):
        a, b = getattr(m_e, f"mmtm{i}"), getattr(m_g, f"mmtm{i}")
        assert a.step == b.step == 9
        torch.testing.assert_close(b.running_avg_weight_visual, a.running_avg_weight_visual, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(b.running_avg_weight_skeleton, a.running_avg_weight_skeleton, rtol=1e-6,
                                   atol=1e-7)
        assert int(b._step_dev.item()) == 9


def test_view_streams_equal_single_stream(monkeypatch):
    """Trunks on two HIP streams (streams.py) == one stream, bit for bit: every
    kernel is deterministic, so any cross-stream race would show up here."""
    dev = torch.device("cuda:0")
    monkeypatch.setenv("GM_VIEW_STREAMS", "0")
    m_1, _, tr_1 = _run(False, 5, dev)
    monkeypatch.setenv("GM_VIEW_STREAMS", "1")
    m_2, _, tr_2 = _run(False, 5, dev)
    assert tr_1 == tr_2
    s1, s2 = m_1.state_dict(), m_2.state_dict()
    for k in s1:
        assert torch.equal(s1[k], s2[k]), k


def _run_gate(device_gate, graphs, steps, dev):
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    torch.manual_seed(0)
    m = MMTM_MVCNN().to(dev)
    gate = Bias_Mitigation_Strong(epsilon=2e-3, curation_windowsize=2, branchnames=["net_view_0", "net_view_1"],
                                  starting_epoch=1)
    # The host-gate run routes its flags through the device gate's select/mask kernels
    # (mask_curation): the host gate's own curated backward skips the substituted
    # modality's excitation GEMMs, a different fp32 summation order whose 1e-8
    # differences flip bf16 activation roundings and decorrelate two runs in a few steps.
    st = BalancedStep(m, lr=0.05, gate=gate, graphs=graphs, device_gate=device_gate)
    assert st.device_gate == device_gate
    if not device_gate:  # host flags through the same select/mask kernels: bitwise comparable
        for i in (2, 3, 4):
            getattr(m, f"mmtm{i}").mask_curation = True
    st.on_epoch_begin(1)
    g = torch.Generator(device=dev).manual_seed(5)
    xs = [torch.randn(4, 2, 3, 64, 64, device=dev, generator=g) for _ in range(3)]
    ys = [torch.randint(0, 40, (4,), device=dev, generator=g) for _ in range(3)]
    trace = []
    for i in range(steps):
        loss = st(xs[i % 3], ys[i % 3])
        if device_gate:
            st.sync_gate()
        trace.append((float(loss), gate.d_BDR, st.flags.curation_mode, st.flags.caring_modality))
    return m, st, trace


@pytest.mark.parametrize("graphs", [False, True])
def test_device_gate_equals_host_gate(graphs):
    """The on-device gate (decision kernel behind the norms+SGD pass, MMTM curation from
    device flags, one graph for every setting) reproduces the host gate step by step:
    decisions, d_BDR, losses, parameters and MMTM running averages."""
    dev = torch.device("cuda:0")
    m_h, st_h, tr_h = _run_gate(False, False, 10, dev)
    m_d, st_d, tr_d = _run_gate(True, graphs, 10, dev)
    assert {t[2] for t in tr_h} == {True, False}, "the trace should contain curation steps"
    if graphs:
        assert len(st_d._graphs) == 1
    diffs = [(a[0] - b[0], a[1] - b[1], a[2], b[2]) for a, b in zip(tr_h, tr_d)]
    for a, b in zip(tr_h, tr_d):
        assert a[2:] == b[2:], diffs
        assert a[0] == pytest.approx(b[0], rel=1e-6, abs=1e-6), diffs
        assert a[1] == pytest.approx(b[1], rel=1e-6, abs=1e-9), diffs
    sh, sd = m_h.state_dict(), m_d.state_dict()
    for k in sh:
        torch.testing.assert_close(sd[k], sh[k], rtol=1e-6, atol=1e-6, msg=k)
    for i in (2, 3, 4):
        a, b = getattr(m_h, f"mmtm{i}"), getattr(m_d, f"mmtm{i}")
        torch.testing.assert_close(b.running_avg_weight_visual, a.running_avg_weight_visual, rtol=1e-6, atol=1e-7)


def test_larger_second_batch_under_capture():
    """a batch larger than every earlier one is captured directly (no eager
    warm-up at its shape), so the BN ticket / split-K turnstile scratch must grow INSIDE the
    capture.  The grown buffers must not replace the eager stream's (their zero fill is only
    recorded): graph steps over growing batches equal eager steps, and an eager step after
    them (the failed-capture fallback's path) still runs on zeroed tickets."""
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    sizes = [2, 2, 8, 8, 16]
    xs = [torch.randn(b, 2, 3, 64, 64, device=dev, generator=g) for b in sizes]
    ys = [torch.randint(0, 40, (b,), device=dev, generator=g) for b in sizes]

    def run(graphs):
        torch.manual_seed(0)
        m = MMTM_MVCNN().to(dev)
        gate = Bias_Mitigation_Strong(epsilon=2e-3, curation_windowsize=2,
                                      branchnames=["net_view_0", "net_view_1"], starting_epoch=1)
        st = BalancedStep(m, lr=0.05, gate=gate, graphs=graphs, device_gate=True)
        st.on_epoch_begin(1)
        losses = [float(st(x, y)) for x, y in zip(xs, ys)]
        assert st.graphs == graphs, "a capture failed and the engine fell back to eager steps"
        st.graphs = False  # one eager step after the captured ones, at the largest shape
        losses.append(float(st(xs[-1], ys[-1])))
        torch.cuda.synchronize()
        return m, losses

    m_e, l_e = run(False)
    m_g, l_g = run(True)
    assert l_g == pytest.approx(l_e, rel=1e-6, abs=1e-6)
    se, sg = m_e.state_dict(), m_g.state_dict()
    for k in se:
        torch.testing.assert_close(sg[k], se[k], rtol=1e-6, atol=1e-6, msg=k)


def test_failed_capture_then_recapture():
    """a capture that grows the BN ticket / split-K turnstile scratch and then fails
    must not leave those buffers (whose zero fill exists only in the dropped graph) for the next
    capture on the same stream; and the failure must not leave the default CUDA generator in its
    capture state.  A failure is injected at the end of the first capture's
    body; the engine falls back to eager steps; graphs are then re-enabled and the step is
    captured again.  Losses and parameters equal an all-eager run."""
    from greedy_multimodal_learning_amd import streams
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(11)
    sizes = [2, 24, 24, 24]  # 24: larger than any batch an earlier test ran, so scratch grows
    xs = [torch.randn(b, 2, 3, 64, 64, device=dev, generator=g) for b in sizes]
    ys = [torch.randint(0, 40, (b,), device=dev, generator=g) for b in sizes]

    def build(graphs):
        torch.manual_seed(0)
        m = MMTM_MVCNN().to(dev)
        gate = Bias_Mitigation_Strong(epsilon=2e-3, curation_windowsize=2,
                                      branchnames=["net_view_0", "net_view_1"], starting_epoch=1)
        st = BalancedStep(m, lr=0.05, gate=gate, graphs=graphs, device_gate=True)
        st.on_epoch_begin(1)
        return m, st

    m_e, st_e = build(False)
    l_e = [float(st_e(x, y)) for x, y in zip(xs, ys)]

    from greedy_multimodal_learning_amd import bn, conv, vtrunk
    caches = (vtrunk._bn_scratch, conv._splitk_ws, bn._scratch)

    def shrink():  # every cached scratch buffer too small for the next call: a capture must grow it
        torch.cuda.synchronize()
        for cache in caches:
            for k in list(cache):
                cache[k] = torch.zeros(16, dtype=torch.uint8, device=dev)

    m_g, st_g = build(True)
    l_g = [float(st_g(xs[0], ys[0]))]  # eager first step (B = 2)
    shrink()
    orig = st_g._fwd_bwd
    injected = []

    def failing(*a):
        out = orig(*a)
        if torch.cuda.is_current_stream_capturing() and not injected:
            injected.append(len(streams._grown_in_capture))
            raise RuntimeError("injected capture failure")
        return out

    st_g._fwd_bwd = failing
    l_g.append(float(st_g(xs[1], ys[1])))  # capture at B = 24 fails -> eager fallback
    assert injected and injected[0] > 0, "no scratch grew inside the failed capture"
    assert st_g.capture_failures and not st_g.graphs
    assert streams._grown_in_capture == []
    cap_key = (0, torch.cuda.graph.default_capture_stream.stream_id)
    assert all(cap_key not in c for c in caches), "scratch grown in the failed capture was kept"
    torch.randn(1, device=dev)  # the default generator is usable outside a capture
    st_g._fwd_bwd = orig
    shrink()  # the retry's capture grows again: under the capture key, with its own recorded fill
    st_g.graphs = True  # the retry: capture again on the same capture stream
    l_g += [float(st_g(x, y)) for x, y in zip(xs[2:], ys[2:])]
    assert st_g.graphs and len(st_g._graphs) == 1
    torch.cuda.synchronize()
    assert l_g == pytest.approx(l_e, rel=1e-6, abs=1e-6)
    se, sg = m_e.state_dict(), m_g.state_dict()
    for k in se:
        torch.testing.assert_close(sg[k], se[k], rtol=1e-6, atol=1e-6, msg=k)


def test_release_rng_capture_state_keeps_the_random_stream():
    """streams.release_rng_capture_state - run by the engine after every failed capture to take
    the default CUDA generator out of the capture state a failed capture leaves it in (the round-5
    "RuntimeError: Off..." of test_xent_bad_label_is_nan) - records one
    capture and never replays it: the default generator's stream of numbers is unchanged.  (A
    deliberately invalidated capture is not used to reproduce the stuck state here: on HIP it
    leaves the process's later HIP calls failing with "operation failed due to a previous error
    during capture".)"""
    from greedy_multimodal_learning_amd.streams import release_rng_capture_state
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    a = torch.rand(1000, device=dev)
    torch.manual_seed(1234)
    release_rng_capture_state(dev)
    b = torch.rand(1000, device=dev)
    assert torch.equal(a, b)
