"""MI355X-native drop-in mirror of the reference package path (see conformer-nemo_amd/README in DESIGN.md)."""
