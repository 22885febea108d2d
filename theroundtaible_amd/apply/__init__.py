"""``roundtable apply``: RTDIFF/1 block edits, scope enforcement, backups, manifest updates."""
