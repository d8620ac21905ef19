"""Mirror of the reference's ``tools`` helpers that sit on the hot path."""
