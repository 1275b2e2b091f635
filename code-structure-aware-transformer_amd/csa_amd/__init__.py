"""csa_amd — MI355X-native CSA-Trans attention hot path.

Public surface:
  csa_amd.module.sbm_attn          SBMAttention, FullAttention, Attention   (module/sbm_attn.py)
  csa_amd.module.STE               SampleGraphSparseGraph                   (module/STE.py)
  csa_amd.module.disentangled_attn DisentangledAttn                         (module/disentangled_attn.py)
  csa_amd.ops                      torch.ops.csa.* custom ops + autograd functions
  csa_amd.data                     synthetic AST batches with the reference's relation encoding
"""
__version__ = "0.1.0"
