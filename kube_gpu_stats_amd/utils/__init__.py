"""Shared helpers: configuration from flags/env, logging, small HTTP client."""
