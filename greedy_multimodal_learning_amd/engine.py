"""Fused balanced training step for MI355X (single GPU or data parallel).

Same sequence and semantics as one iteration of the reference's
`Model_.train_loop` (src/framework.py:307-322) with the guided gate:

    zero_grad -> forward(curation flags) -> blend_loss -> backward
    -> [DP: gradient all-reduce] -> on_backward_end (gating) -> SGD.step

re-organised for the hardware:

* all parameters live in ONE flat fp32 buffer and all gradients in another
  (parameters are views), laid out in reverse registration order so that
  gradients become ready front-to-back during backward;
* gradient all-reduce (RCCL over xGMI) runs per ~`bucket_mb` bucket from
  post-accumulate-grad hooks, overlapping the rest of backward;
* the per-branch norm pass of the gate and the SGD update are ONE HIP pass
  (`gm_group_sumsq` with lr != 0): it reads every parameter before updating
  it, so the sums equal those `compute_BDR` takes before `optimizer.step()`;
  the only host sync per step is the 8-double copy the gate needs for its
  decision (the decision applies to the NEXT forward, as in the reference);
* the trunk runs in bf16 (autocast) on channels_last activations; master
  weights, gradients, the MMTM FC chain and all reductions stay fp32;
* `graphs=True`: after one eager step, each curation setting
  (none / caring 0 / caring 1 ...) is captured ONCE as a hipGraph of the whole
  step - zero_grad, forward, loss, backward, fused norms+SGD - and replayed;
  the host then only copies the 8 group sums and runs the gate's decision.
  Everything the step mutates lives in device memory (parameters, BN running
  statistics and counters, MMTM running averages and their step counter), so a
  replay is exactly an eager step; the host-side `step` attributes of the MMTM
  modules are advanced by the engine after each replay.
"""
import os

import torch
import torch.distributed as dist

from .callbacks import GroupNorms
from .gradsink import GradSink
from .losses import blend_loss
from .streams import alias_capture_stream, all_side_streams, capture_dropped, capture_replayed, \
    release_rng_capture_state, side_stream
from .streams import enabled as streams_enabled
from .vtrunk import drop_pending_wgrads


_DEBUG_BUCKETS = os.environ.get("GM_DEBUG_BUCKETS", "0") == "1"

# RCCL channels bound = CUs reserved for RCCL's kernels beside the spin hand-off kernels.
RCCL_CHANNELS_DEFAULT = 64


# hardware queues a data-parallel rank needs: the trunk stream, the weight-gradient stream, the
# gradient-bucket (comm) stream and RCCL's own stream must not share a queue - a stream queued
# behind a long RCCL kernel on a shared queue stalls (test_gpu_rccl_residency.py measured 393 ms
# behind a CU-holding kernel at HIP's default of 4); 8 leaves headroom (the pool's cap is 32)
DP_HW_QUEUES = 8


def check_hw_queues():
    """Warn when a data-parallel engine runs with fewer than DP_HW_QUEUES hardware queues.
    GPU_MAX_HW_QUEUES is read once, when the HIP runtime initialises - set it before the first
    HIP call of the rank (bench.py does, before importing torch)."""
    try:
        q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        q = 4
    if q < DP_HW_QUEUES:
        import warnings
        warnings.warn(f"data-parallel BalancedStep with GPU_MAX_HW_QUEUES={q} (< {DP_HW_QUEUES}): the trunk, "
                      "weight-gradient, gradient-bucket and RCCL streams share hardware queues and can stall "
                      "behind each other; export GPU_MAX_HW_QUEUES=8 before the rank's first HIP call",
                      RuntimeWarning, stacklevel=3)
    return q


def bound_rccl_channels():
    """Bound RCCL's channel count (NCCL_MAX_NCHANNELS) before any communicator of this
    process exists, unless the user set it: an RCCL collective kernel runs one workgroup
    per channel, so the bound is exactly the number of CUs its kernels can hold while they
    overlap backward.  RCCL reads the variable at communicator creation; bench.py calls
    this before init_process_group, the engine again before it creates its own group.
    Returns the bound."""
    return int(os.environ.setdefault("NCCL_MAX_NCHANNELS", str(RCCL_CHANNELS_DEFAULT)))


def rccl_reserved_cus():
    """CUs the residency plan keeps free for RCCL: the channel bound (NCCL_MAX_NCHANNELS),
    or GM_RCCL_RESERVED_CUS when the operator overrides it."""
    if "GM_RCCL_RESERVED_CUS" in os.environ:
        return int(os.environ["GM_RCCL_RESERVED_CUS"])
    return bound_rccl_channels()


class _Flags:
    """Holds the curation flags like the reference's Model_ (src/framework.py:137-138)."""

    def __init__(self):
        self.curation_mode = False
        self.caring_modality = None
        self.stop_training = False  # set by CompletedStopping / a NaN loss (src/framework.py:321-322)


class FlatParams:
    """All parameters of `model` as views of ONE flat fp32 buffer and their
    gradients as views of a second one (same offsets), in the order backward produces
    the gradients (model.grad_order(), else reverse registration order).  Conv weights
    keep the model's memory format (KRSC when channels_last)."""

    def __init__(self, model, channels_last=False):
        self.device = next(model.parameters()).device
        order = getattr(model, "grad_order", None)
        # the model's backward-production order when it states one (model.grad_order: views
        # interleaved per layer), else reverse registration order
        params = list(order()) if callable(order) else [p for _, p in model.named_parameters()][::-1]
        assert len(params) == len(list(model.parameters())), "grad_order must list every parameter once"
        total = sum(p.numel() for p in params)
        self.param = torch.empty(total, device=self.device, dtype=torch.float32)
        self.grad = torch.zeros(total, device=self.device, dtype=torch.float32)
        self.slices = {}
        off = 0
        for p in params:
            n = p.numel()
            view = self.param[off:off + n]
            if p.dim() == 4 and channels_last:
                O, I, kh, kw = p.shape
                nhwc = view.view(O, kh, kw, I)
                nhwc.copy_(p.data.permute(0, 2, 3, 1))
                p.data = nhwc.permute(0, 3, 1, 2)
                p.grad = self.grad[off:off + n].view(O, kh, kw, I).permute(0, 3, 1, 2)
            else:
                view.copy_(p.data.reshape(-1))
                p.data = view.view(p.shape)
                p.grad = self.grad[off:off + n].view(p.shape)
            self.slices[p] = (off, n)
            off += n
        self.total = total


class GradBuckets:
    """Bucketed gradient all-reduce overlapped with backward.

    The flat gradient buffer is cut into contiguous ~bucket_mb slices; a
    post-accumulate-grad hook counts the parameters of each bucket and launches
    an async all_reduce(SUM) on the slice the moment its last gradient lands,
    while autograd keeps producing the next ones.  `finish()` launches any bucket
    a parameter without gradient left incomplete and waits for all of them.
    Backend-agnostic: RCCL ("nccl") on the GPU, gloo in the CPU tests."""

    def __init__(self, flat, process_group=None, bucket_mb=25.0):
        self.flat = flat
        self.pg = process_group
        cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        order = sorted(flat.slices.items(), key=lambda kv: kv[1][0])
        self.buckets = []
        cur, start, end = [], 0, 0
        for p, (off, n) in order:
            if cur and (off + n - start) > cap:
                self.buckets.append((start, end, cur))
                cur = []
            if not cur:
                start = off
            cur.append(p)
            end = off + n
        if cur:
            self.buckets.append((start, end, cur))
        self.deferred = False
        self.names = {}
        self.bucket_of = {}
        for bi, (_, _, ps) in enumerate(self.buckets):
            for p in ps:
                self.bucket_of[p] = bi
                p.register_post_accumulate_grad_hook(self._on_grad)
        self.reset()

    def reset(self):
        self._pending = [len(ps) for (_, _, ps) in self.buckets]
        self._seen = set()
        self._via_sink = set()
        self._first = {}
        self._works = []
        g = self.flat.grad
        # the step's compute streams: main (current at step start) + the trunks' side
        # streams; a bucket's gradients may come from any of them
        self._streams = ([torch.cuda.current_stream(g.device)] + all_side_streams(g.device)) if g.is_cuda else []
        if g.is_cuda and getattr(self, "_comm", None) is None:
            self._comm = torch.cuda.Stream(device=g.device)

    def _on_grad(self, p):
        """post-accumulate-grad hook.  torch fires it even when the backward returned
        None for the parameter, i.e. also right after a HIP kernel delivered that
        gradient in place through the sink (_on_sink): those calls are not a second
        gradient and are skipped."""
        if self.deferred or id(p) in self._via_sink:
            return
        self._count(p)

    def _on_pending(self, p):
        """p's in-place delivery is deferred (gradsink.sink_pending): skip its hook."""
        if not self.deferred:
            self._via_sink.add(id(p))

    def _on_sink(self, p):
        """a HIP backward wrote p's gradient straight into the flat buffer (gradsink)."""
        if self.deferred:  # a hipGraph capture: the step reduces after the replay
            return
        self._count(p)
        self._via_sink.add(id(p))

    def _count(self, p):
        bi = self.bucket_of[p]
        if id(p) in self._seen:
            first = self._first.get(id(p), "")
            raise RuntimeError(f"gradient of parameter {self.names.get(id(p), tuple(p.shape))} delivered twice "
                               f"in one step (used twice under data parallelism){first}")
        self._seen.add(id(p))
        if _DEBUG_BUCKETS:
            import traceback
            self._first[id(p)] = "\nfirst delivery:\n" + "".join(traceback.format_stack(limit=12))
        if self._pending[bi] == -1:
            raise RuntimeError("gradient delivered after its bucket was all-reduced "
                               f"(a parameter used twice in one step under data parallelism: {tuple(p.shape)})")
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi):
        s, e, _ = self.buckets[bi]
        t = self.flat.grad[s:e]
        if self._streams:
            # issue from a comm stream that waits for every compute stream, so the
            # collective sees gradients written on any of them
            comm = self._comm
            for st in self._streams:
                comm.wait_stream(st)
            with torch.cuda.stream(comm):
                self._works.append(dist.all_reduce(t, group=self.pg, async_op=True))
        else:
            self._works.append(dist.all_reduce(t, group=self.pg, async_op=True))
        self._pending[bi] = -1

    def finish(self):
        for bi, c in enumerate(self._pending):
            if c != -1:
                self._launch(bi)
        for w in self._works:
            w.wait()
        self._works = []

    def reduce_all(self):
        """All buckets at once, after a replayed hipGraph step produced every gradient
        (collectives stay outside the graph: RCCL work is issued eagerly on the comm
        stream behind the replay)."""
        self.reset()
        self.finish()


class BalancedStep:
    def __init__(self, model, lr=0.1, gate=None, compute_dtype=torch.bfloat16, channels_last=True,
                 process_group=None, bucket_mb=25.0, branchnames=("net_view_0", "net_view_1"),
                 MMTMnames=("visual", "skeleton"), graphs=False, device_gate=None, dp_buckets=None):
        self.model = model
        self.lr = float(lr)
        self.gate = gate
        self.compute_dtype = compute_dtype
        self.channels_last = channels_last
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if process_group is not None else 1
        self.flags = _Flags()
        self.device = next(model.parameters()).device
        if channels_last:
            model.to(memory_format=torch.channels_last)
        named = list(model.named_parameters())
        self.flat = FlatParams(model, channels_last)
        self._seed = torch.ones((), device=self.device, dtype=torch.float32)  # backward seed
        if self.device.type == "cuda":  # the fused head backward's zero rows, outside any capture
            from .head import zero_row
            for name, mod in model.named_modules():
                if name.endswith("fc") and isinstance(mod, torch.nn.Linear):
                    zero_row(self.device, mod.in_features)
        self.flat_grad = self.flat.grad
        if self.device.type == "cuda" and streams_enabled():
            for i in range(int(getattr(model, "num_views", 2)) - 1):
                side_stream(self.device, i)  # created up front: the DP buckets wait on them
        if self.device.type == "cuda":
            from . import vtrunk
            vtrunk._wgrad_stream(self.device)  # (the stacked trunk's weight-gradient stream, likewise)
        self.norms = GroupNorms(named, list(branchnames), list(MMTMnames))
        if gate is not None:
            gate.set_model(model, ignore=False)
            gate.set_model_pytoune(self.flags)
            gate.on_train_begin({})
        self.buckets = None
        # dp_buckets (default: world > 1) - True also on a one-rank group, so the bucketed
        # collective path (and its graph capture) runs on a single GPU (tests)
        if (self.world > 1) if dp_buckets is None else (bool(dp_buckets) and process_group is not None):
            for m in model.modules():
                if hasattr(m, "zero_grads_for_curated"):
                    m.zero_grads_for_curated = True  # every bucket fills every step
            self.buckets = GradBuckets(self.flat, process_group, bucket_mb)
            self.buckets.names = {id(p): n for n, p in named}
        # HIP conv/BN backward kernels write their parameter gradients straight into
        # the flat buffer (no AccumulateGrad add) and fire the bucket hook themselves
        # lazy_zero: no zero-fill of the flat gradient buffer per step (gradsink.py)
        self.sink = GradSink(self.flat.slices.keys(),
                             on_ready=self.buckets._on_sink if self.buckets is not None else None,
                             lazy_zero=True)
        if self.buckets is not None:
            self.sink.on_pending = self.buckets._on_pending
        self.last_loss = None
        self.last_outs = None  # the last step's branch logits (fp32), e.g. for training accuracy
        self.step_count = 0
        self.timer = None  # optional (start_event, end_event) list collector for the fused pass
        self.wprep = None
        if self.device.type == "cuda" and channels_last and compute_dtype == torch.bfloat16:
            from .conv import WeightPrep
            self.wprep = WeightPrep(model)
        # graphs under data parallelism: the per-rank compute (zero_grad, forward, loss,
        # backward) is ONE hipGraph; the gradient all-reduce and the fused norms+SGD pass
        # run eagerly behind each replay (no collective inside a graph)
        self.graphs = bool(graphs) and self.device.type == "cuda"
        # DP + graphs: with RCCL ("nccl") the bucketed all-reduces are captured INSIDE the
        # step's graph on the comm stream, each bucket forked off backward the moment its
        # last gradient is written, so the replay overlaps the collectives with the rest of
        # backward (north_star: all-reduce overlapped with backward).  gloo collectives
        # cannot be captured: there (and with GM_DP_GRAPH_COLLECTIVES=0) the per-rank
        # compute is the graph and the all-reduce + norms/SGD run eagerly behind it.
        self.graph_collectives = False
        self._capture_pg = None
        if self.buckets is not None and self.device.type == "cuda":
            check_hw_queues()
        if self.buckets is not None and self.graphs:
            backend = dist.get_backend(process_group)
            self.graph_collectives = (backend == "nccl"
                                      and os.environ.get("GM_DP_GRAPH_COLLECTIVES", "1") != "0")
            if self.graph_collectives:
                bound_rccl_channels()
                # the captured all-reduces run on a process group of their own that never
                # issues an eager collective: its communicator is initialised here (device_id:
                # eager connect, no work item), so the group's watchdog never holds an event
                # recorded on the stream being captured (HIP refuses that query and the
                # watchdog aborts the process).  The eager steps keep using `process_group`.
                # new_group is collective over the default group: every rank builds the engine.
                self._capture_pg = dist.new_group(ranks=dist.get_process_group_ranks(process_group),
                                                  backend="nccl", device_id=self.device)
        if self.device.type == "cuda":
            self._plan_residency(model)
        self._graphs = {}
        self._gpool = None
        self.capture_failures = []  # messages of failed captures (each one fell back, see __call__)
        self._static = None
        self._slots = {}
        from .balanced_mmtm import MMTM_mitigate
        from .mmtm_n import MMTM_N
        self._mmtms = [m for m in model.modules() if isinstance(m, (MMTM_mitigate, MMTM_N))]
        # on-device gate: the Strong gate's decision made by a kernel behind
        # the norms+SGD pass and consumed by the MMTM kernels from device memory, so no
        # host sync per step and one graph for every curation setting
        # Two branches over MMTM_mitigate: gm_gate_state (the reference's d = BDR_0 - BDR_1);
        # N branches over MMTM_N (C4 / C5): gm_gate_state_n (the host gate's N-branch rule,
        # callbacks.bdr_decision), up to GATE_MAX_BRANCHES branches.
        from . import _lib as L
        from .callbacks import Bias_Mitigation_Strong
        nb = len(gate.branchnames) if isinstance(gate, Bias_Mitigation_Strong) else 0
        two = (nb == 2 and bool(self._mmtms)
               and all(isinstance(m, MMTM_mitigate) and not m.SEonly for m in self._mmtms))
        many = (2 <= nb <= L.GATE_MAX_BRANCHES and bool(self._mmtms)
                and all(isinstance(m, MMTM_N) and m.N == nb for m in self._mmtms))
        eligible = self.device.type == "cuda" and (two or many)
        if device_gate is None:
            import os as _os
            device_gate = _os.environ.get("GM_DEVICE_GATE", "1") != "0"
        self.device_gate = bool(device_gate) and eligible
        self.gate_n = self.device_gate and not two
        self.gate_state = None
        if self.device_gate:
            st = L.GateStateN() if self.gate_n else L.GateState()
            if self.gate_n:
                st.nb = nb
            st.caring = -1
            st.window = int(gate.curation_windowsize)
            st.eps = float(gate.epsilon)
            st.unlock = int(bool(getattr(gate, "unlock", False)))
            self.gate_state = torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(self.device)
            for m in self._mmtms:
                m.device_gate = self.gate_state

    def _plan_residency(self, model):
        """The library's device residency plan (gm_set_residency): launches whose
        workgroups wait on each other (single-launch BatchNorm, split-K turnstile) size
        their grids for the trunk streams that run at once, the ranks sharing this GPU
        (found by exchanging (host, device) over the step's group) and, under RCCL data
        parallelism, the CUs the all-reduce kernels hold while they overlap backward:
        RCCL's channel bound (rccl_reserved_cus: one workgroup per channel)."""
        from . import _lib as L
        views = int(getattr(model, "num_views", 2))
        streams = views if streams_enabled() else 1
        from . import vtrunk
        if vtrunk.ENABLED and hasattr(model, "_forward_stacked") and self.compute_dtype == torch.bfloat16:
            # the view-batched trunk: grouped launches on one stream (+ its weight gradients);
            # no view streams, so the single-launch BatchNorm may size its grid for that
            # (GM_BN_FUSE_STREAMS, when set, keeps the operator's value)
            streams = 2 if vtrunk.WGRAD_STREAM else 1
            if "GM_BN_FUSE_STREAMS" not in os.environ:
                from .streams import set_concurrency
                set_concurrency(streams)
        sharers, reserved = 1, 0
        if self.pg is not None and self.world > 1:
            import socket
            me = (socket.gethostname(), torch.cuda.get_device_properties(self.device).uuid
                  if hasattr(torch.cuda.get_device_properties(self.device), "uuid") else self.device.index)
            who = [None] * self.world
            dist.all_gather_object(who, (me[0], str(me[1])), group=self.pg)
            sharers = sum(1 for w in who if w == (me[0], str(me[1])))
        if self.buckets is not None and dist.get_backend(self.pg) == "nccl":
            reserved = rccl_reserved_cus()
        self.residency = L.set_residency(streams=max(1, streams), sharers=max(1, sharers), reserved_cus=reserved)

    # ---------------- on-device gate ----------------
    def _sums_and_gate(self):
        """The fused norms+SGD pass; with the on-device gate its step rides in the same finalize
        launch (gm_group_sumsq_gate)."""
        if self.device_gate:
            return self.norms.sums(grad_scale=1.0 / self.world, lr=self.lr, gate=self.gate_state,
                                   gate_n=self.gate_n)
        return self.norms.sums(grad_scale=1.0 / self.world, lr=self.lr)

    def gate_struct(self):
        """The device gate state as its ctypes mirror (GateState / GateStateN); a host sync."""
        from . import _lib as L
        cls = L.GateStateN if self.gate_n else L.GateState
        return cls.from_buffer_copy(self.gate_state.cpu().numpy().tobytes())

    def set_gate_struct(self, st):
        """Write a (modified) gate_struct() back to the device."""
        self.gate_state.copy_(torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8))

    def sync_gate(self):
        """Copy the device gate state to the host mirrors (gate.d_BDR, its M
        accumulators, curation_step, the flags object); returns it as a dict.  The
        only host sync of the on-device gate, taken when someone asks.  Also raises
        GreedyMMLError if a fused BatchNorm / split-K hand-off timed out since the
        last call (gm_device_faults)."""
        from . import _lib as L
        L.check_device_faults()  # a timed-out in-launch hand-off since the last sync raises here
        if not self.device_gate:
            return None
        st = self.gate_struct()
        g, fl = self.gate, self.flags
        g.d_BDR = float(st.d_bdr)
        if self.gate_n:
            nb = int(st.nb)
            g.M_bypass = [float(v) for v in st.M_bypass[:nb]]
            g.M_main = [float(v) for v in st.M_main[:nb]]
            g.BDR = [float(v) for v in st.bdr[:nb]]
            if nb == 2:  # the two-branch host mirrors, as the host gate keeps them
                g.M_bypass_modal_0, g.M_bypass_modal_1 = g.M_bypass
                g.M_main_modal_0, g.M_main_modal_1 = g.M_main
        else:
            g.M_bypass_modal_0, g.M_bypass_modal_1 = float(st.M[0]), float(st.M[1])
            g.M_main_modal_0, g.M_main_modal_1 = float(st.M[2]), float(st.M[3])
        g.curation_step = int(st.curation_step)
        fl.curation_mode = bool(st.curation_mode)
        fl.caring_modality = None if st.caring < 0 else int(st.caring)
        return {"curation_mode": fl.curation_mode, "caring_modality": fl.caring_modality, "d_BDR": g.d_BDR,
                "curation_step": g.curation_step, "n_curated": int(st.n_curated)}

    # ---------------- the step ----------------
    def forward(self, x, mean=True):
        fl = self.flags
        self.model._no_mean = not mean
        try:
            with torch.autocast("cuda", dtype=self.compute_dtype, enabled=self.compute_dtype != torch.float32):
                return self.model(x, curation_mode=fl.curation_mode, caring_modality=fl.caring_modality)
        finally:
            self.model._no_mean = False

    def _fwd_bwd(self, x, y):
        if not self.sink.lazy_zero:
            self.flat_grad.zero_()
        if self.buckets is not None:
            self.buckets.reset()
        drop_pending_wgrads()
        self.sink.begin_step()
        wp = self.wprep
        try:
            if wp is not None:
                wp.run()  # bf16 copies of every conv weight, one launch
                wp.activate()
            _, outs, _, _ = self.forward(x, mean=False)
            if wp is not None:
                wp.deactivate()
            outs = [o.float() for o in outs]
            loss = blend_loss(outs, y)
            # the backward seed from a persistent ones tensor made before any capture (no
            # fill launch per step; blend_loss returns a 0-d fp32 loss)
            if getattr(self, "_seed", None) is None or self._seed.shape != loss.shape \
                    or self._seed.device != loss.device or self._seed.dtype != loss.dtype:
                self._seed = torch.ones_like(loss)
            loss.backward(self._seed)
            if self.device.type == "cuda":
                # backward nodes of the side-stream trunks ran on their streams (some of
                # them write gradients in place, outside autograd's leaf-stream sync)
                cur = torch.cuda.current_stream(self.device)
                for s in all_side_streams(self.device):
                    cur.wait_stream(s)
        except BaseException:
            drop_pending_wgrads()
            raise
        finally:
            self.sink.end_step()
            if wp is not None:
                wp.deactivate()
        if self.buckets is not None and not self.buckets.deferred:
            self.buckets.finish()
        return loss, [o.detach() for o in outs]

    def _graph_key(self):
        if self.device_gate:
            return ("device-gate", self.lr)
        fl = self.flags
        return (bool(fl.curation_mode), fl.caring_modality if fl.curation_mode else None, self.lr)

    def bind_batches(self, *pairs):
        """Register device batches (x, y) as static graph inputs.  A step on a bound
        batch replays that slot's own graph and copies nothing; a loader refills a slot
        in place while another slot's step runs (double-buffered input).  Any other
        batch is copied into the engine's own static buffers first, as before."""
        self._slots = {(x.data_ptr(), y.data_ptr()): (x, y) for x, y in pairs}

    def _slot_of(self, x, y):
        # data parallel: no bound slots, so the graph-cache key (curation setting, lr) is the
        # same on every rank - a rank that captures (with its collective agreement) while
        # another replays would hang; the lr is rank-identical (one schedule on every rank)
        if self.world > 1:
            return None
        slot = self._slots.get((x.data_ptr(), y.data_ptr())) if self._slots else None
        if slot is None or slot[0].shape != x.shape or slot[0].stride() != x.stride() or slot[0].dtype != x.dtype \
                or slot[1].shape != y.shape or slot[1].dtype != y.dtype:
            return None
        return slot

    def _capture(self, key, inputs=None):
        """Record one whole step for the current curation flags (nothing executes)."""
        steps = [(m, m.step) for m in self._mmtms]
        g = torch.cuda.CUDAGraph()
        if self._gpool is None:
            self._gpool = torch.cuda.graph_pool_handle()
        torch.cuda.synchronize(self.device)
        dp = self.buckets is not None
        inline = dp and self.graph_collectives  # collectives captured in the graph
        if inline:
            self.buckets.pg = self._capture_pg  # (see __init__: no eager work on this group)
        if dp and not inline:
            self.buckets.deferred = True
        # thread_local: the process group's watchdog thread keeps querying its events
        # while this thread captures (global mode would invalidate the capture)
        mode = "thread_local" if dp else "global"
        eager_sid = torch.cuda.current_stream(self.device).stream_id
        try:
            with torch.cuda.graph(g, pool=self._gpool, capture_error_mode=mode):
                alias_capture_stream(self.device.index if self.device.index is not None
                                     else torch.cuda.current_device(), eager_sid)
                loss, outs = self._fwd_bwd(*(inputs or self._static))
                loss = loss.detach()
                sums = None if (dp and not inline) else self._sums_and_gate()
        finally:
            if dp:
                self.buckets.deferred = False
                self.buckets.pg = self.pg
            for m, st in steps:  # capture ran the Python forward but no kernel
                m.step = st
                m._step_mirror = st
        self._graphs[key] = (g, loss, sums, outs)
        return self._graphs[key]

    def __call__(self, x, y):
        """One balanced step on batch (x [B,V,3,H,W], y [B]); returns the loss tensor
        (with graphs=True: the captured step's static loss tensor)."""
        self.model.train(True)
        gate = self.gate
        if self.graphs and self.step_count > 0:
            slot = self._slot_of(x, y)
            if slot is None:
                st = self._static
                if st is None or st[0].shape != x.shape or st[1].shape != y.shape or st[0].dtype != x.dtype:
                    if self._graphs:  # (as above: no graph destroyed under a running replay)
                        torch.cuda.synchronize(self.device)
                    self._graphs = {}
                    # the destroyed graphs released the private pool; capturing into a released
                    # pool trips the caching allocator (use_count == 0): start a fresh one
                    self._gpool = None
                    self._static = st = (x.detach().clone(), y.detach().clone())
                else:
                    if st[0].data_ptr() != x.data_ptr():
                        st[0].copy_(x)
                    if st[1].data_ptr() != y.data_ptr():
                        st[1].copy_(y)
            key = (self._graph_key(), None if slot is None else (x.data_ptr(), y.data_ptr()))
            entry, err = self._graphs.get(key), None
            if entry is None:
                # a learning-rate change (ReduceLROnPlateau) makes the old-lr graphs dead weight;
                # the last replay may still be running: destroy nothing before it is done
                stale = [k for k in self._graphs if k[0][-1] != self.lr]
                if stale:
                    torch.cuda.synchronize(self.device)
                for k in stale:
                    del self._graphs[k]
                if stale and not self._graphs:
                    self._gpool = None  # (every graph of the pool destroyed: a fresh pool)
                try:
                    entry = self._capture(key, slot)
                except RuntimeError as e:  # capture refused on this system
                    entry, err = None, e
                    self.capture_failures.append(str(e))
                    capture_dropped()  # (scratch grown in the failed capture was never zeroed)
                    try:
                        release_rng_capture_state(self.device)
                    except RuntimeError as e2:  # best effort: the fallback below still runs
                        self.capture_failures.append(f"release_rng_capture_state: {e2}")
                if self.buckets is not None and self.world > 1 and not self._agree(entry is not None):
                    # every rank takes the same fallback, so the ranks' collective sequences
                    # stay identical (a rank replaying in-graph collectives beside one that
                    # reduces eagerly would hang or sum the wrong buffers)
                    self._graphs.pop(key, None)
                    capture_dropped()
                    entry = None
                    err = err or RuntimeError("graph capture failed on another rank")
            if entry is None:
                import sys
                if self.graph_collectives:  # first fall back to the collectives-outside-the-graph form
                    print(f"[greedy_multimodal_learning_amd] capturing the all-reduce failed ({err}); "
                          "collectives run eagerly behind each replay", file=sys.stderr, flush=True)
                    self.graph_collectives = False
                    self._graphs = {}
                    self._gpool = None
                    torch.cuda.synchronize(self.device)
                    return self(x, y)
                print(f"[greedy_multimodal_learning_amd] hipGraph capture failed ({err}); eager steps from now on",
                      file=sys.stderr, flush=True)
                self.graphs = False
                self._graphs = {}
                torch.cuda.synchronize(self.device)
                return self(x, y)
            g, loss, sums, outs = entry
            want = gate is not None and hasattr(gate, "needs_bdr") and gate.needs_bdr()
            g.replay()
            capture_replayed()
            if self.buckets is not None and not self.graph_collectives:
                self.buckets.reduce_all()
                sums = self._sums_and_gate()
            for m in self._mmtms:
                m.step += 1
                m._step_mirror = m.step
            self.last_outs = outs  # the graph's static branch logits, current after the replay
            return self._after(loss, sums, want)
        # detached: a kept-alive autograd graph would pin AccumulateGrad nodes to this
        # step's stream (breaks later graph capture, and holds memory)
        loss, self.last_outs = self._fwd_bwd(x, y)
        loss = loss.detach()
        want = gate is not None and hasattr(gate, "needs_bdr") and gate.needs_bdr()
        t = self.timer
        if t is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        sums = self._sums_and_gate()
        if t is not None:
            ev1.record()
            t.append((ev0, ev1))
        return self._after(loss, sums, want)

    def _agree(self, ok):
        """True iff `ok` on every rank (an eager MIN all-reduce on the step's group)."""
        on_dev = dist.get_backend(self.pg) == "nccl"
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.pg)
        return bool(int(t.item()))

    def _after(self, loss, sums, want):
        gate = self.gate
        if gate is not None and not self.device_gate:
            if want:
                gate.pending_sums = sums
            gate.on_backward_end(self.step_count)
            gate.pending_sums = None
        self.last_loss = loss
        self.step_count += 1
        return loss

    def on_epoch_begin(self, epoch):
        if self.gate is not None:
            self.gate.on_epoch_begin(epoch, {})
            if self.device_gate:  # push the unlock flag (int at byte offset 12)
                flag = torch.tensor([int(bool(getattr(self.gate, "unlock", False)))], dtype=torch.int32)
                self.gate_state[12:16].copy_(flag.view(torch.uint8))
