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


class GradSink:
    def __init__(self, params, on_ready=None):
        self.params = list(params)
        self.on_ready = on_ready
        self.active = False
        self._written = set()
        for p in self.params:
            p._gm_sink = self

    def begin_step(self):
        self._written = set()
        self.active = True

    def end_step(self):
        self.active = False

    def detach(self):
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
