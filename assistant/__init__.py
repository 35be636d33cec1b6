"""assistant -- Telegram / REST assistant-bot framework with a RAG pipeline, served by the MI355X engine.

Django apps: assistant.ai, assistant.bot, assistant.rag, assistant.storage, assistant.processing,
assistant.loading, assistant.broadcasting, assistant.admin (same module paths and public APIs as the
reference framework).  The framework-agnostic core (ai providers, utils, RAG aggregation, bot domain,
Telegram formatting) imports without Django; ORM / admin / REST / Celery modules need Django.
"""
__version__ = "0.1.0"
