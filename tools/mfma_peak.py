"""Sustained bf16 MFMA rate of this MI355X under full load (tools/native/mfma_peak.hip:
back-to-back v_mfma_f32_32x32x16_bf16 on registers, every CU busy), against the 2.5 PFLOP/s
datasheet peak - the practical ceiling for the trunk kernels.  Build: see tools/native/build.sh."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "native", "mfma_peak.so"))
    dev = torch.device("cuda:0")
    out = torch.zeros(1024, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    for mode, what in ((0, "constant operands"), (1, "random operands, fixed"), (2, "random operands, changing")):
      for threads in (256, 512):
        for mult in (1, 2):
            blocks, iters = cus * mult, 2000
            lib.mfma_peak_launch(ctypes.c_void_p(out.data_ptr()), blocks, threads, iters, mode, st)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                lib.mfma_peak_launch(ctypes.c_void_p(out.data_ptr()), blocks, threads, iters, mode, st)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 5 / 1e3
            flops = blocks * (threads // 64) * iters * 8 * 32 * 32 * 16 * 2
            print(f"{what}: {blocks} blocks x {threads} threads: {t * 1e6:.1f} us, {flops / t / 1e12:.0f} TFLOP/s "
                  f"= {flops / t / 2.5e15:.3f} of 2.5 PF; implied clock {flops / t / (cus * 4 * 32768 / 32) / 1e9:.2f} GHz",
                  flush=True)


if __name__ == "__main__":
    main()
