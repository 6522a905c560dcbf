"""icap — MI355X-native (gfx950) prefix image-captioning hot path.

Drop-in for the device hot path of thenoobychocobo/gpt2-image-captioning
(src/models.py, src/train.py, src/embeddings/clip.py, src/embeddings/vit.py): all arithmetic runs in
the hand-written HIP kernels of libicap_hip.so (include/icap.h); PyTorch only
owns device memory, streams, graphs and torch.distributed.
"""

__version__ = "0.1.0"

from .clip import CLIPVisionConfig, CLIPVisionTower, extract_clip_embedding_from_image, extract_clip_embeddings, load_clip_model  # noqa: E402,F401
from .dataset import CocoDataset, SyntheticCaptionDataset  # noqa: E402,F401
from .engine import CaptionTrainer  # noqa: E402,F401
from .gpt2 import GPT2Config, GPT2LMHeadModel  # noqa: E402,F401
from .mapper import MLPMappingNetwork, TransformerMappingNetwork  # noqa: E402,F401
from .models import ImageCaptioningModel, load_gpt2_tokenizer  # noqa: E402,F401
from .train import train  # noqa: E402,F401
from .vit import ViTConfig, ViTImageTower, extract_vit_embedding_from_image, extract_vit_embeddings, load_vit_model  # noqa: E402,F401
from .dino import (DINOv3ImageTower, DinoConfig, extract_dino_embeddings, get_dinov3_preprocessor,  # noqa: E402,F401
                   load_dinov3_models)
