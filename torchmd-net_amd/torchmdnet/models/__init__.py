__all__ = ["equivariant-transformer", "tensornet"]
