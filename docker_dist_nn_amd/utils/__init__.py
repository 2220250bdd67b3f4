from .native import native, native_available, native_path

__all__ = ["native", "native_available", "native_path"]
