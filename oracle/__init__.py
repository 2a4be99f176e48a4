"""TEST INFRASTRUCTURE ONLY: CPU restatement of the reference checksum path (parity checker)."""
