"""Console output (chalk/ora replacement). Colors only on a TTY; ``quiet`` silences everything."""
from __future__ import annotations

import os
import sys
from typing import Optional, TextIO

_CODES = {"bold": "1", "dim": "2", "red": "31", "green": "32", "yellow": "33", "blue": "34",
          "magenta": "35", "cyan": "36", "white": "37", "gray": "90"}
KNIGHT_COLORS = {"Claude": "38;2;217;119;6", "Gemini": "38;2;59;130;246", "GPT": "38;2;16;185;129"}


class UI:
    def __init__(self, stream: Optional[TextIO] = None, quiet: bool = False, color: Optional[bool] = None):
        self.stream = stream or sys.stdout
        self.quiet = quiet
        if color is None:
            color = hasattr(self.stream, "isatty") and self.stream.isatty() and not os.environ.get("NO_COLOR")
        self.color = color

    def paint(self, text: str, *styles: str) -> str:
        if not self.color or not styles:
            return text
        codes = ";".join(KNIGHT_COLORS.get(s) or _CODES.get(s, "") for s in styles)
        return f"\x1b[{codes}m{text}\x1b[0m"

    def knight(self, name: str, text: Optional[str] = None) -> str:
        return self.paint(text if text is not None else name, name if name in KNIGHT_COLORS else "white")

    def print(self, text: str = "", *styles: str) -> None:
        if not self.quiet:
            print(self.paint(text, *styles), file=self.stream, flush=True)

    def dim(self, t: str) -> None:
        self.print(t, "dim")

    def warn(self, t: str) -> None:
        self.print(t, "yellow")

    def error(self, t: str) -> None:
        self.print(t, "red")

    def ok(self, t: str) -> None:
        self.print(t, "green")


NULL_UI = UI(quiet=True)
