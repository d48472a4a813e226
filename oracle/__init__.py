"""CPU oracle for the balanced multi-modal training step.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package
(`greedy_multimodal_learning_amd/`) imports this package.  Only `tests/`,
`__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py` may use it,
and there only as the checker / the timed CPU baseline, never as the thing
measured on the GPU.

What it is: an independent fp32 PyTorch-CPU + numpy restatement of the
reference's hot path (SebastianHafner/greedy_multimodal_learning):

* `resnet_ref`  - the torchvision ResNet-18/50 architecture the reference calls
                  (`src/model.py:53-56`; torchvision itself is not vendored and
                  not installed here).
* `mmtm_ref`    - `MMTM_mitigate.forward` in all modes (`src/balanced_mmtm.py:49-154`).
* `model_ref`   - `MMTM_MVCNN` (`src/model.py:15-108`).
* `gating_ref`  - `compute_BDR` and the `Bias_Mitigation_Strong/Random` state
                  machines (`src/callbacks.py:173-302`), `blend_loss`/`acc`
                  (`train.py:23-40`).
* `step_ref`    - one training step in the reference order
                  (`src/framework.py:307-322`), the CPU baseline.
* `weights`     - a seeded numpy (PCG64) parameter generator so that fixtures
                  need not carry 95 MB state dicts.

Parity pinning: `tests/golden/*.npz` were produced by importing the reference
itself (with dependency shims) in the build container; the generating script is
`tests/golden/make_golden.py`.  `tests/test_oracle_golden.py` checks this
oracle against those fixtures.  The trunk arithmetic of torchvision is pinned
only through this restatement (torchvision is unpinned upstream, README.md:8).
"""
