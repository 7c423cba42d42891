"""CPU oracle (test infrastructure; see ripple_oracle.h)."""
