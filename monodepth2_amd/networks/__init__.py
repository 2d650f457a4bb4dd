"""networks/* API of the reference (networks/__init__.py): PyTorch-ROCm modules."""
from .resnet_encoder import ResnetEncoder
from .decoders import DepthDecoder, PoseDecoder, PoseCNN

__all__ = ["ResnetEncoder", "DepthDecoder", "PoseDecoder", "PoseCNN"]
