"""Package logger; same logger name as the reference (pynbodyext/log.py:4)."""
import logging

logger = logging.getLogger("pynext")
