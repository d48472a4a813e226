"""In-place parameter-gradient delivery for the HIP autograd functions.

PyTorch delivers a parameter gradient by handing the tensor a backward returns
to AccumulateGrad, which adds it into `param.grad` (one extra elementwise kernel
and a full read+write of the gradient per parameter per step).  When the engine
owns the gradients (one flat fp32 buffer, zeroed at the start of each step) the
HIP kernels can write the gradient straight into `param.grad` instead:

    sink = GradSink(params, on_ready=buckets_hook)   # engine, once
    sink.begin_step()                                  # engine, each step
    ...
    tgt = sink_target(p)        # HIP function backward: (grad_tensor, accumulate) or None
    <kernel writes / adds into tgt[0]>
    sink_done(p)                # fires the same hook post-accumulate-grad would
    return None                 # for that parameter

The first write of a step overwrites (the buffer was zeroed anyway), any later
use of the same parameter in the same step accumulates, so modules shared
between branches stay correct.  Parameters outside a sink (or a sink that is
not active) keep the ordinary autograd path.
"""

import torch


class GradSink:
    """lazy_zero: the caller does NOT zero the gradients before the step.  A gradient
    that autograd is about to accumulate into is zeroed first (tensor pre-hook, only
    for parameters not yet written this step), and end_step() zeroes the gradients
    nothing wrote; sink writes overwrite anyway.  With every gradient sink-delivered
    (the HIP training step) no zero-fill of the gradient buffer runs at all."""

    def __init__(self, params, on_ready=None, lazy_zero=False):
        self.params = list(params)
        self.on_ready = on_ready
        self.on_pending = None  # a delivery that will be reported later (sink_pending)
        self.active = False
        self.lazy_zero = lazy_zero
        self._written = set()
        self._hooks = []
        for p in self.params:
            p._gm_sink = self
            if lazy_zero:
                self._hooks.append(p.register_hook(lambda g, p=p: self._before_accumulate(p)))

    def _before_accumulate(self, p):
        if self.active and id(p) not in self._written:
            self._written.add(id(p))
            if p.grad is not None:
                p.grad.zero_()

    def begin_step(self):
        self._written = set()
        self.active = True

    def end_step(self):
        if self.active and self.lazy_zero:
            rest = [p.grad for p in self.params if id(p) not in self._written and p.grad is not None]
            if rest:
                torch._foreach_zero_(rest)
        self.active = False

    def detach(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for p in self.params:
            if getattr(p, "_gm_sink", None) is self:
                del p._gm_sink
        self.params = []
        self.active = False


def sink_target(p):
    """(gradient tensor to write, accumulate flag) if `p`'s gradient is delivered
    in place this step, else None."""
    s = getattr(p, "_gm_sink", None)
    if s is None or not s.active or p.grad is None:
        return None
    key = id(p)
    acc = key in s._written
    s._written.add(key)
    return p.grad, acc


def sink_done(p):
    s = p._gm_sink
    if s.on_ready is not None:
        s.on_ready(p)


def sink_pending(p):
    """p's gradient will be written in place by a launch issued later in this backward
    (vtrunk's batched weight gradients): its autograd hook is not a delivery, sink_done
    follows once the launch is issued."""
    s = p._gm_sink
    if s.on_pending is not None:
        s.on_pending(p)


class GradJoin:
    """Gradient of ONE activation consumed by several HIP backward functions (the
    ResNet block input: the first convolution and the identity / downsample branch).

    Autograd would materialise each consumer's gradient and add them with an extra
    elementwise kernel.  Instead each consumer, in its backward, calls
    `contribute(compute)`: every consumer but the last stores its gradient as the
    pending addend and returns None to autograd; the last one computes its gradient
    WITH the pending addend folded in (the conv dgrad epilogue adds it:
    gm_conv2d_dgrad_add_bf16) and returns the total.  Order-independent; a consumer
    that cannot fold gets `addend` and must add it itself."""

    def __init__(self):
        self.n = 0
        self.done = 0
        self.pending = None
        # every consumer that may come last accepts a MaskedAddend (the view-batched trunk's
        # identity blocks: vtrunk.vblock sets it)
        self.masked_ok = False

    def register(self):
        self.n += 1

    def first_of_many(self):
        """True when the next contribution is stored as the pending addend (not the last)."""
        return self.pending is None and self.done + 1 < self.n

    def contribute(self, compute):
        self.done += 1
        add, self.pending = self.pending, None
        g = compute(add)
        if self.done >= self.n:
            self.done = 0
            return g
        self.pending = g
        return None


class MaskedAddend:
    """A pending join addend kept as (dy, 1-bit mask): dz = dy where the mask bit is set - the
    identity branch's gradient of a block-output ReLU, which the consuming convolution's dgrad
    epilogue forms itself (gm_conv2d_dgrad_grouped_masked_bf16) instead of reading a dres tensor
    that the BatchNorm backward would have written."""

    def __init__(self, dy, mask):
        self.dy = dy
        self.mask = mask
