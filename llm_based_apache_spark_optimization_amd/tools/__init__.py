"""Command-line tools (manual API client)."""
