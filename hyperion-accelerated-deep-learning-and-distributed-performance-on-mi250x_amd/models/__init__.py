"""Model zoo (reference C5, C14-C17, C26): torchvision/HF-key-compatible definitions."""
from .resnet import ResNet, create_resnet50, resnet18, resnet34, resnet50  # noqa: F401
