"""nlspn_eccv20_amd — MI355X-native (gfx950) NLSPN non-local spatial propagation.

The hot path of XJTUXYC/NLSPN_ECCV20 (src/model/nlspnmodel.py:179-381 and the DCNv2
forward it calls) as hand-written HIP kernels behind a C ABI (include/nlspn_prop.h),
with a torch-facing mirror of the reference interface:

  propagation.affinity_normalization / off_insert / prop_step / propagate
  propagation.propagate_normalized — the loop from prologued planes (heads.head_epilogue_prologue)
  heads                         — the decoder's last three convs as one kernel (+ the fused prologue)
  ops                           — the same kernels as torch.ops.nlspn.* operators
  propagation.PropagationPlan   — the whole section as one native hipGraph
  propagation.NLSPNPropagation  — nn.Module with the reference's state_dict names
  dcn                           — `DCN`-compatible module (seam 2)
  model.NLSPNModel              — the whole reference model (seam 1), encoder/decoder on MIOpen
  model.SectionGraph            — its propagation section (GRU mode included) as one hipGraph
  replay                        — the reference's summary dumps (offset.npy / aff.npy / gamma.npy) re-run
"""
from .model import NLSPNModel, SectionGraph
from .propagation import (NLSPNPropagation, PropagationPlan, affinity_normalization, kernel_geometry,
                          off_insert, prop_step, propagate, propagate_normalized)

__all__ = ["NLSPNModel", "NLSPNPropagation", "PropagationPlan", "SectionGraph", "affinity_normalization",
           "kernel_geometry", "off_insert", "prop_step", "propagate", "propagate_normalized"]
__version__ = "0.1.0"
