"""Sandboxed read-only shell tool for ``verify_commands`` (`src/utils/verify.ts:8-174`).

Same whitelist, forbidden patterns and limits: 5 s timeout, 1 MB output buffer,
5,000-char result, <= 4 commands per call, secrets stripped from the environment.
"""
from __future__ import annotations

import os
import re
import subprocess
from typing import Callable, Iterable, List, Optional

WHITELISTED = frozenset({"ls", "cat", "head", "tail", "grep", "find", "wc", "file", "stat",
                         "sort", "uniq", "basename", "dirname"})
FORBIDDEN_PATTERNS = [
    (re.compile(r";"), ";"),
    (re.compile(r"`"), "`"),
    (re.compile(r"\$\("), r"\$\("),
    (re.compile(r"\$\{"), r"\$\{"),
    (re.compile(r"&&"), "&&"),
    (re.compile(r"\|\|"), r"\|\|"),
    (re.compile(r"-exec\b"), r"-exec\b"),
    (re.compile(r"-delete\b"), r"-delete\b"),
    (re.compile(r"-ok\b"), r"-ok\b"),
    # fix over the reference: find's other action / write primaries (-execdir, -okdir run programs;
    # -fprint, -fprint0, -fprintf, -fls write files)
    (re.compile(r"(?<![\w-])-(?:exec|ok)\w+"), r"-exec*/-ok*"),
    (re.compile(r"(?<![\w-])-f(?:print\w*|ls)\b"), r"-fprint*/-fls"),
]
FORBIDDEN_COMMANDS = frozenset({
    "rm", "mv", "cp", "chmod", "chown", "chgrp", "curl", "wget", "eval", "source", "node", "python",
    "python3", "ruby", "perl", "php", "bash", "sh", "zsh", "npm", "npx", "yarn", "pnpm", "pip", "apt",
    "brew", "dd", "mkfs", "mount", "umount", "kill", "pkill", "ssh", "scp", "rsync", "nc", "ncat", "telnet",
})
SENSITIVE_ENV = ("OPENAI_API_KEY", "ANTHROPIC_API_KEY", "GEMINI_API_KEY", "GOOGLE_API_KEY",
                 "AWS_SECRET_ACCESS_KEY", "AWS_ACCESS_KEY_ID", "GITHUB_TOKEN", "GH_TOKEN", "NPM_TOKEN",
                 "CLAUDECODE")
TIMEOUT_S = 5.0
MAX_BUFFER = 1024 * 1024
MAX_OUTPUT = 5000


def validate_command(command: str) -> Optional[str]:
    """None if allowed, else the rejection reason.

    Deliberate fix over the reference (`src/utils/verify.ts:55-98`): a newline / carriage return
    or a lone ``&`` also separates commands under ``bash -c``, so both are rejected too (the
    reference passes ``"ls\\nrm -rf x"`` and ``"ls & rm x"``)."""
    cmd = command.strip()
    if not cmd:
        return "empty command"
    for pat, src in FORBIDDEN_PATTERNS:
        if pat.search(cmd):
            return f"forbidden pattern: {src}"
    if "\n" in cmd or "\r" in cmd:
        return "forbidden pattern: newline (command separator)"
    if re.search(r"(?<![&>])&(?!&|1)", cmd.replace("2>&1", "")):
        return "forbidden pattern: & (background / separator)"
    rest = re.sub(r"2>\s*/dev/null", "", cmd).replace("2>&1", "")
    if ">>" in rest:
        return "forbidden pattern: append redirect (>>)"
    if ">" in rest:
        return "forbidden pattern: output redirect (>)"
    if "<" in rest:
        return "forbidden pattern: input redirect (<)"
    placeholder = "\x00ESCAPED_PIPE\x00"
    segments = [s.replace(placeholder, "\\|").strip() for s in cmd.replace("\\|", placeholder).split("|")]
    for seg in segments:
        if not seg:
            return "empty pipe segment"
        base = seg.split()[0] if seg.split() else ""
        if not base:
            return "empty segment"
        if base in FORBIDDEN_COMMANDS:
            return f"forbidden command: {base}"
        if base not in WHITELISTED:
            return f"command not whitelisted: {base}"
    return None


def _sanitized_env() -> dict:
    env = dict(os.environ)
    for k in SENSITIVE_ENV:
        env.pop(k, None)
    return env


def execute_command(command: str, root: str, env: Optional[dict] = None) -> str:
    try:
        r = subprocess.run(["bash", "-c", command], cwd=root, env=env or _sanitized_env(),
                           capture_output=True, timeout=TIMEOUT_S)
    except subprocess.TimeoutExpired:
        return f"### VERIFY: {command}\n```\n[TIMEOUT after 5s]\n```"
    out = r.stdout[:MAX_BUFFER].decode("utf-8", "replace").strip()
    err = r.stderr[:MAX_BUFFER].decode("utf-8", "replace").strip()
    trunc = out[:MAX_OUTPUT] + "\n...(truncated)" if len(out) > MAX_OUTPUT else out
    if r.returncode != 0:
        combined = trunc or err or f"exit code {r.returncode}"
        return f"### VERIFY: {command}\n```\n{combined}\n```"
    return f"### VERIFY: {command}\n```\n{trunc or '(empty output)'}\n```"


def resolve_verify_commands(commands: Iterable[str], root: str,
                            log: Optional[Callable[[str], None]] = None) -> str:
    env = _sanitized_env()
    results: List[str] = []
    for c in list(commands)[:4]:
        c = str(c)
        err = validate_command(c)
        if err:
            results.append(f"### VERIFY: {c}\n```\n[DENIED] {err}\n```")
            if log:
                log(f"  [DENIED] {c} — {err}")
            continue
        if log:
            log(f"  Running: {c}")
        results.append(execute_command(c, root, env))
    return "\n\n".join(results)
