"""mift.apps: reference-compatible entry points (W1..W6)."""
