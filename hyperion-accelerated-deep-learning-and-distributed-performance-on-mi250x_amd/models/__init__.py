"""Model zoo (reference C5, C14-C17, C26): torchvision/HF-key-compatible definitions."""
from .llama import LlamaConfig, LlamaForCausalLM, llama2_7b  # noqa: F401
from .resnet import ResNet, create_resnet50, resnet18, resnet34, resnet50  # noqa: F401
from .simple_lm import GPT2_PAD, GPT2_VOCAB, SimpleTransformerLM, gpt2_small_lm, simple_lm_256, simple_lm_768  # noqa: F401
from .transformer import CustomTransformer, TransformerEncoder, TransformerEncoderLayer, create_custom_transformer  # noqa: F401
from .vit import VisionTransformer, create_vit_model, fallback_cnn, vit_b_16, vit_tiny  # noqa: F401
