from .read_write import FORMATS, read, write

__all__ = ["FORMATS", "read", "write"]
