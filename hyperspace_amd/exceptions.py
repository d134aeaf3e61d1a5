"""Domain exceptions (reference ``HyperspaceException.scala:19``, ``actions/NoChangesException.scala:29``)."""


class HyperspaceException(Exception):
    def __init__(self, msg: str):
        super().__init__(msg)
        self.msg = msg


class NoChangesException(HyperspaceException):
    """Signals a no-op action; ``Action.run`` logs it and returns instead of failing."""
