from .ingress import LayerClient, StageFailure, serve
from .proto import METHOD, Matrix, Row

__all__ = ["LayerClient", "StageFailure", "serve", "METHOD", "Matrix", "Row"]
