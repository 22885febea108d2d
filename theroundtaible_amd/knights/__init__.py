"""Knight backends (reference layer L2): engine-hosted models, scripted fakes, registry."""
from .base import KnightBackend, TurnRequest, TurnResult
from .fake import FakeBackend, consensus_reply
