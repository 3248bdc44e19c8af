"""ASR collection mirror: only the Conformer encoder plugin path."""
