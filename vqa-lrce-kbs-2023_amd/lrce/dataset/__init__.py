from .synthetic import SyntheticQADataset  # noqa: F401
