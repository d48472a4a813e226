"""greedy_multimodal_learning_amd - MI355X-native balanced multi-modal training step.

Drop-in modules mirroring the reference (SebastianHafner/greedy_multimodal_learning):

* `model.MMTM_MVCNN`             <- src/model.py
* `balanced_mmtm.MMTM_mitigate`  <- src/balanced_mmtm.py (+ get_rescale_weights)
* `callbacks.Bias_Mitigation_Strong / _Random` <- src/callbacks.py gating
* `losses.blend_loss / acc`      <- train.py:23-40
* `engine.BalancedStep`          fused step (flat params, fused BDR+SGD, DP reducer)

Kernels: libgreedymml_hip.so (C ABI: include/greedymml.h), built with
`python -m greedy_multimodal_learning_amd.build`.
"""
__version__ = "0.1.0"
