from .log import get_logger, LOG_FORMAT

__all__ = ["get_logger", "LOG_FORMAT"]
