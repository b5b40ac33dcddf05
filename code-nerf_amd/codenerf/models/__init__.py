from .model import CodeNeRFModel, ShapeTextureEmbedding, get_params_tensor  # noqa: F401
