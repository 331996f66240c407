"""MI355X-native learned-image-codec hot path (drop-in for the TF2 encode/decode surface of
AlexFuster/Neural_network_image_compression).

Public surface:
  Encoder, Decoder, ProClass  -- mirror tf2_0/src/{encoder,decoder,utils}.py
  Codec                       -- one device context (torch.uint8 cuda tensors in/out)
  weights                     -- layer table, seeded init, safetensors checkpoints
"""
from . import weights  # noqa: F401

__all__ = ["Encoder", "Decoder", "ProClass", "Codec", "weights", "latent_shape"]


def __getattr__(name):
    # the codec classes pull in torch + the HIP library lazily
    if name in ("Encoder", "Decoder", "ProClass", "Codec"):
        from . import codec

        return getattr(codec, name)
    if name == "latent_shape":
        from ._lib import latent_shape

        return latent_shape
    raise AttributeError(name)
