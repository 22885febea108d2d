"""Chronicle (`src/utils/chronicle.ts:8-54`): the project's append-only decision log."""
from __future__ import annotations

import os
from typing import Iterable

from ..utils.atomic import atomic_write_text, file_lock, read_text

# Header written by `init` (init.ts:406-410). The reference's first *append* into a
# missing file uses a different (Dutch) header (chronicle.ts:38); we keep that quirk.
INIT_HEADER = "# Chronicle — TheRoundtAIble\n\nThe record of all decisions made at this table.\n\n---\n\n"
APPEND_HEADER = "# Chronicle - TheRoundtAIble\n\nBeslissingen log van dit project.\n\n---\n\n"


def read_chronicle(project_root: str, chronicle_path: str) -> str:
    p = os.path.join(project_root, chronicle_path)
    return read_text(p) if os.path.exists(p) else ""


def render_entry(topic: str, outcome: str, knights: Iterable[str], date: str) -> str:
    return "\n".join([f"## {date} — {topic}", "", f"**Knights:** {', '.join(knights)}", "",
                      outcome, "", "---", ""])


def append_to_chronicle(project_root: str, chronicle_path: str, *, topic: str, outcome: str,
                        knights: Iterable[str], date: str) -> None:
    p = os.path.join(project_root, chronicle_path)
    with file_lock(p):
        content = read_text(p) if os.path.exists(p) else APPEND_HEADER
        atomic_write_text(p, content + render_entry(topic, outcome, knights, date))
