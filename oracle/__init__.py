"""ORACLE / TEST INFRASTRUCTURE package (CPU restatement of the reference hot path)."""
