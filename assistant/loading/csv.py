"""Reference import path ``assistant.loading.csv`` (kept for API compatibility)."""
from assistant.loading.csv_loader import COLUMNS_COUNT, CSVLoader, normalize_title, read_rows  # noqa: F401
