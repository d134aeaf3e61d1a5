"""Explain display modes and the highlight-aware buffer (reference
``plananalysis/DisplayMode.scala:24-89``, ``plananalysis/BufferStream.scala:23-83``)."""
from __future__ import annotations

from ..index import constants as C


class Tag:
    def __init__(self, open_: str, close: str):
        self.open = open_
        self.close = close


class DisplayMode:
    new_line = "\n"
    begin_end_tag = Tag("", "")
    highlight_tag = Tag("", "")


class PlainTextMode(DisplayMode):
    def __init__(self, highlight: Tag = None):
        self.highlight_tag = highlight if highlight and (highlight.open or highlight.close) \
            else Tag("<----", "---->")


class HTMLMode(DisplayMode):
    new_line = "<br>"
    begin_end_tag = Tag("<pre>", "</pre>")

    def __init__(self, highlight: Tag = None):
        self.highlight_tag = highlight if highlight and (highlight.open or highlight.close) \
            else Tag('<b style="background:LightGreen">', "</b>")


class ConsoleMode(DisplayMode):
    def __init__(self, highlight: Tag = None):
        self.highlight_tag = highlight if highlight and (highlight.open or highlight.close) \
            else Tag("\u001b[42m", "\u001b[0m")


def get_display_mode(conf) -> DisplayMode:
    tag = Tag(conf.get(C.HIGHLIGHT_BEGIN_TAG, ""), conf.get(C.HIGHLIGHT_END_TAG, ""))
    mode = conf.get(C.DISPLAY_MODE, C.DisplayMode.PLAIN_TEXT).lower()
    if mode == C.DisplayMode.HTML:
        return HTMLMode(tag)
    if mode == C.DisplayMode.CONSOLE:
        return ConsoleMode(tag)
    return PlainTextMode(tag)


class BufferStream:
    def __init__(self, mode: DisplayMode):
        self.mode = mode
        self._buf = []

    def write(self, s: str = "") -> "BufferStream":
        self._buf.append(s)
        return self

    def write_line(self, s: str = "") -> "BufferStream":
        self._buf.append(s + self.mode.new_line)
        return self

    def highlight(self, s: str) -> "BufferStream":
        """Wrap in highlight tags, keeping leading/trailing whitespace outside the tags."""
        stripped = s.strip()
        if not stripped:
            self._buf.append(s)
            return self
        lead = s[:len(s) - len(s.lstrip())]
        trail = s[len(s.rstrip()):]
        self._buf.append(f"{lead}{self.mode.highlight_tag.open}{stripped}"
                         f"{self.mode.highlight_tag.close}{trail}")
        return self

    def with_tag(self) -> str:
        return self.mode.begin_end_tag.open + "".join(self._buf) + self.mode.begin_end_tag.close

    def __str__(self):
        return "".join(self._buf)
