"""docker_dist_nn_amd — a layer-pipelined MLP training and inference engine for AMD MI355X.

A from-scratch, MI355X-native framework with the capabilities of
TollanBerhanu/docker-dist-nn (a fully-connected network split layer-wise across a chain of
gRPC workers): each stage of ``layer_distribution`` runs on its own GPU process, activations
and gradients move between stages over RCCL (xGMI) instead of protobuf/gRPC, the per-layer
compute is hand-written gfx950 HIP (MFMA GEMMs with fused epilogues, fused softmax-CE and
optimizers), and the reference's JSON model/topology schema, per-stage weight files and
``run_grpc_fcnn.py`` / ``run_grpc_inference.py`` entry points stay compatible.

Subpackages: ``models`` (MLP specs), ``ops`` (kernel wrappers + torch references),
``parallel`` (comm backends, PPxDP groups, pipeline schedules), ``engine`` (stages, trainer,
inference), ``serve`` (gRPC compat ingress), ``utils``.
"""
import torch  # noqa: F401  -- load torch's HIP runtime before our extension

__version__ = "0.1.0"

from .models import MLPSpec, LayerSpec, NAMED_MODELS  # noqa: E402

__all__ = ["MLPSpec", "LayerSpec", "NAMED_MODELS", "__version__"]
