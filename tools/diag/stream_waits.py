"""Python-level cross-stream synchronisation of one eager bench step: every
Stream.wait_stream / wait_event, Event.record / wait and Tensor.record_stream call with
the streams involved and the calling line, in issue order (autograd's C++ engine syncs
are not visible here).  usage: python tools/diag/stream_waits.py [batch]"""
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
LOG = []
ON = [False]


def site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "greedy_multimodal_learning_amd" in fr.filename or "tools/" in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
    return "?"


def sid(s):
    return getattr(s, "stream_id", "?")


def patch():
    S, E = torch.cuda.Stream, torch.cuda.Event
    ws, we, er, ew, rs = S.wait_stream, S.wait_event, E.record, E.wait, torch.Tensor.record_stream

    def wait_stream(self, other):
        if ON[0]:
            LOG.append(f"wait_stream  {sid(self)} <- {sid(other)}  {site()}")
        return ws(self, other)

    def wait_event(self, ev):
        if ON[0]:
            LOG.append(f"wait_event   {sid(self)}  {site()}")
        return we(self, ev)

    def record(self, stream=None):
        if ON[0]:
            LOG.append(f"event.record {sid(stream or torch.cuda.current_stream())}  {site()}")
        return er(self, stream)

    def ewait(self, stream=None):
        if ON[0]:
            LOG.append(f"event.wait   {sid(stream or torch.cuda.current_stream())}  {site()}")
        return ew(self, stream)

    def record_stream(self, stream):
        if ON[0]:
            LOG.append(f"record_stream {sid(stream)} {tuple(self.shape)}  {site()}")
        return rs(self, stream)
    S.wait_stream, S.wait_event, E.record, E.wait = wait_stream, wait_event, record, ewait
    torch.Tensor.record_stream = record_stream


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    patch()
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    dev = torch.device("cuda:0")
    m = MMTM_MVCNN().to(dev)
    gate = Bias_Mitigation_Strong(epsilon=0.01, curation_windowsize=5, branchnames=["net_view_0", "net_view_1"],
                                  starting_epoch=1)
    st = BalancedStep(m, lr=0.1, gate=gate, graphs=False)
    st.on_epoch_begin(1)
    x = torch.randn(2, b, 224, 224, 3, device=dev).bfloat16().permute(1, 0, 4, 2, 3)
    y = torch.randint(0, 40, (b,), device=dev)
    st(x, y)
    torch.cuda.synchronize()
    ON[0] = True
    st(x, y)
    ON[0] = False
    torch.cuda.synchronize()
    print(f"main stream {torch.cuda.current_stream().stream_id}")
    for line in LOG:
        print(line)


if __name__ == "__main__":
    main()
