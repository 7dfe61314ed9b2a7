"""Metric data model."""
