from .operator import denormalize, integrate, normalize, resize, scale, warp, warp_grid

__all__ = ["denormalize", "integrate", "normalize", "resize", "scale", "warp", "warp_grid"]
