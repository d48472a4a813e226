"""Per-view HIP streams for the unshared trunks.

The reference runs its two ResNet trunks one after the other on one stream
(src/model.py:65-106).  The trunks are independent between the MMTM sites, so
here view i > 0 runs on its own HIP stream: small-map layers (layer3/4, their
BatchNorms) of the two views then fill the 256 CUs together instead of leaving
most of them idle.  PyTorch's autograd runs every backward node on the stream
its forward ran on, so backward overlaps the same way; the engine's whole-step
hipGraph capture records the fork/join edges as graph dependencies.

    vs = ViewStreams.for_tensor(x, n_views)     # None on CPU / when disabled
    vs.fork()                                   # side streams wait for main
    f1 = vs.run(1, trunk_1, x1)                 # enqueued on side stream 0
    ...
    vs.join([f1])                               # main waits; f1 recorded on main

Disable with GM_VIEW_STREAMS=0 (A/B measurements).
"""
import os

import torch

_side = {}


def enabled():
    return os.environ.get("GM_VIEW_STREAMS", "1") != "0"


def side_stream(device, i):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, i)
    s = _side.get(key)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _side[key] = s
    return s


# capture stream id -> the stream the step ran on before the capture (engine._capture): the
# per-stream scratch caches (BN tickets, split-K turnstiles: zeroed once) then serve the
# captured step from the buffers the eager warm-up steps created, instead of allocating
# and zero-filling new ones inside the graph (a fill replayed every step)
_capture_alias = {}


def scratch_key(idx):
    """(device, stream) key of the per-stream scratch caches, capture streams aliased."""
    sid = torch.cuda.current_stream(idx).stream_id
    return (idx, _capture_alias.get((idx, sid), sid))


def alias_capture_stream(idx, eager_sid):
    """Inside a capture: the current (capture) stream shares eager_sid's scratch buffers."""
    _capture_alias[(idx, torch.cuda.current_stream(idx).stream_id)] = eager_sid


def zeroed_scratch(cache, device, need, size_of):
    """The per-stream zero-initialised scratch buffer (uint8) of `cache` with >= need bytes.

    Keyed by scratch_key: a capture stream reuses the eager stream's buffer when it is big
    enough.  A buffer that must GROW inside a capture is never put under the aliased key - its
    torch.zeros is only recorded into the graph, not run, so eager launches (a failed capture's
    fallback) would then meet ticket words nobody zeroed; it goes under the capture stream's
    own key instead, where the recorded fill runs before every use."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = scratch_key(idx)
    buf = cache.get(key)
    if buf is not None and buf.numel() >= need:
        return buf
    capturing = torch.cuda.is_current_stream_capturing()
    if capturing:
        key = (idx, torch.cuda.current_stream(idx).stream_id)
        buf = cache.get(key)
        if buf is not None and buf.numel() >= need:
            return buf
    buf = torch.zeros(size_of(buf), device=device, dtype=torch.uint8)
    cache[key] = buf
    if capturing:
        _grown_in_capture.append((cache, key, buf))
    return buf


# buffers grown inside a capture whose graph has not been replayed yet: their zero fill exists
# only as a node of that graph.  If the capture fails or its graph is dropped unreplayed, a later
# capture on the same (default capture) stream would find them big enough and record no fill -
# its BN tickets / split-K turnstiles would start on memory nobody zeroed.
_grown_in_capture = []


def capture_dropped():
    """The capture that grew scratch buffers failed, or its graph is dropped before any replay:
    evict those buffers, so the next capture grows (and zero-fills) its own."""
    for cache, key, buf in _grown_in_capture:
        if cache.get(key) is buf:
            del cache[key]
    _grown_in_capture.clear()


def capture_replayed():
    """A graph holding the recorded fills has run: the grown buffers are zeroed (every kernel
    using them leaves its tickets re-zeroed), so later captures may reuse them without a fill."""
    _grown_in_capture.clear()


_repair_stream = {}


def release_rng_capture_state(device):
    """After a failed capture, end the default generator's capture state.

    torch.cuda.CUDAGraph.capture_begin puts the default CUDA generator into its capture state
    (capture_prologue) BEFORE it asks the allocator for the private pool and begins the stream
    capture, and only capture_end's epilogue takes it out again - after hipStreamEndCapture
    succeeded.  A capture refused in capture_begin after the prologue, or invalidated in its body,
    therefore leaves the generator believing it is captured, and the next eager
    random op anywhere in the process raises "Offset increment outside graph capture
    encountered unexpectedly" (the round-5 test_xent_bad_label_is_nan failure).  One complete
    capture of a trivial kernel on a private stream runs prologue + epilogue and restores it;
    the graph is never replayed, so the generator's offset does not move."""
    g = torch.cuda.CUDAGraph()
    s = _repair_stream.get(device)
    if s is None:  # one private stream for the process (a new stream per call would shift HIP's
        s = _repair_stream[device] = torch.cuda.Stream(device=device)  # stream-to-queue mapping)
    t = torch.zeros(1, device=device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        g.capture_begin()
        try:
            t.add_(1)
        finally:
            g.capture_end()
    torch.cuda.current_stream(device).wait_stream(s)
    del g


def all_side_streams(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return [s for (d, _), s in sorted(_side.items(), key=lambda kv: kv[0]) if d == idx]


_bn_concurrency = [4]  # the library's default (gm_bn_set_concurrency)


def reserve_concurrency(n):
    """Tell the single-launch BatchNorm planner that up to n of its launches may run at
    once (gm_bn_set_concurrency); only ever raised, so co-residency holds for every
    model in the process."""
    if n > _bn_concurrency[0]:
        from . import _lib as L
        L.check(L.load().gm_bn_set_concurrency(int(n)), "gm_bn_set_concurrency")
        _bn_concurrency[0] = n


def set_concurrency(n):
    """Set the single-launch BatchNorm concurrency outright (the engine's view-batched
    trunk: one trunk stream); a later ViewStreams still raises it for its streams."""
    from . import _lib as L
    L.check(L.load().gm_bn_set_concurrency(int(n)), "gm_bn_set_concurrency")
    _bn_concurrency[0] = int(n)


class ViewStreams:
    def __init__(self, device, n):
        reserve_concurrency(n + 2)  # one fused BN per view stream + headroom (RCCL, copies)
        self.device = device
        self.main = torch.cuda.current_stream(device)
        self.side = [side_stream(device, i) for i in range(n - 1)]

    @classmethod
    def for_tensor(cls, x, n):
        if n < 2 or not x.is_cuda or not enabled():
            return None
        return cls(x.device, n)

    def stream(self, i):
        return self.main if i == 0 else self.side[i - 1]

    def fork(self, tensors=()):
        """Side streams wait for everything enqueued on main so far; `tensors`
        (main-stream outputs the side streams will read) are marked in use there."""
        for s in self.side:
            s.wait_stream(self.main)
        for i, t in tensors:
            if i > 0 and t is not None:
                t.record_stream(self.side[i - 1])

    def join(self, tensors=()):
        """Main waits for every side stream; `tensors` produced on side streams
        are marked in use on main."""
        for s in self.side:
            self.main.wait_stream(s)
        for t in tensors:
            if t is not None:
                t.record_stream(self.main)

    def run(self, i, fn, *args):
        if i == 0:
            return fn(*args)
        with torch.cuda.stream(self.side[i - 1]):
            return fn(*args)
