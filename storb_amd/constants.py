"""Piece-size policy constants, as /root/reference/storb/constants.py:11-21."""

MIN_PIECE_SIZE = 16 * 1024  # 16 KiB            (constants.py:11)
MAX_PIECE_SIZE = 256 * 1024 * 1024  # 256 MiB   (constants.py:12)
PIECE_LENGTH_SCALING = 0.5  # (constants.py:13)
PIECE_LENGTH_OFFSET = 8.39  # (constants.py:14)
MAX_UPLOAD_SIZE = 1 * 1024 * 1024 * 1024 * 1024  # 1 TiB (constants.py:16)

# defined but unused by the reference (constants.py:20-21); kept for import parity
EC_DATA_SIZE = 4
EC_PARITY_SIZE = 2

# APDP challenge system (constants.py:28-32)
DEFAULT_RSA_KEY_SIZE = 2048
G_CANDIDATE_RETRY = 1000  # retries for the generator g
S_CANDIDATE_RETRY = 1000  # retries for the challenge secret s
