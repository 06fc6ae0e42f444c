"""HiveQL-subset SQL frontend (N7)."""
from .executor import Session, SQLError  # noqa: F401
