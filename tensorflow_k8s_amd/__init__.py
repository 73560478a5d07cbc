"""tensorflow_k8s_amd (tfk): an MI355X-native TFJob training operator + runtime.

Control plane: C++ (cpp/) TFJob operator, single-node API server, gang scheduler and node agent.
Data plane: this package -- flat-arena graph executor over hand-written gfx950 HIP kernels
(tensorflow_k8s_amd/_C), MultiWorkerMirrored / ParameterServer strategies over RCCL, TF-layout
checkpoints, models (LeNet, ResNet-50/101/152, BERT, Transformer).
"""
__version__ = "0.1.0"
