from .flow2rgb import METHODS, colorwheel, flow2rgb

__all__ = ["METHODS", "colorwheel", "flow2rgb"]
