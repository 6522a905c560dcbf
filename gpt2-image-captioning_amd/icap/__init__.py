"""icap — MI355X-native (gfx950) prefix image-captioning hot path.

Drop-in for the device hot path of thenoobychocobo/gpt2-image-captioning
(src/models.py, src/train.py, src/embeddings/clip.py): all arithmetic runs in
the hand-written HIP kernels of libicap_hip.so (include/icap.h).
"""

__version__ = "0.1.0"
