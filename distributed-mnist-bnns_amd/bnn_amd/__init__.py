"""bnn_amd -- MI355X-native binarized-network training hot path.

Layers: ``functional`` (libbnn.so ops + autograd Functions), ``nn`` (BinarizeLinear /
BinarizeConv2d modules with the reference's ``weight.org`` protocol), ``parallel`` (RCCL
bucketed gradient exchange), ``optim`` (fused latent Adam + clamp), ``nets`` / ``trainer``
(the reference's training loop restated), ``data`` (synthetic MNIST + sampler).
"""
__version__ = "0.1.0"
