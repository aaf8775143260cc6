"""I/O, generators, golden models, timers and configuration."""
