"""Persistence layer for the `.roundtable/` shared brain (reference layer L1)."""
from .session import (create_session, write_discussion, write_decisions, update_status, read_status,
                      list_sessions, find_latest_session, append_round_entry, load_round_entries,
                      append_metrics, render_discussion, render_decisions, slugify)
from .chronicle import read_chronicle, append_to_chronicle
from .manifest import (read_manifest, write_manifest, add_manifest_entry, deprecate_feature,
                       check_manifest, manifest_summary, topic_to_feature_id, feature_summary)
from .decree_log import (read_decree_log, add_decree_entry, active_decrees, format_decrees_for_prompt)
