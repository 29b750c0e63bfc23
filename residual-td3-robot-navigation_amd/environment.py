"""Import shim: `from environment import Environment` (robot-learning.py:14) resolves to the
MI355X drop-in when this directory is first on sys.path."""
from nav.environment import Environment  # noqa: F401
