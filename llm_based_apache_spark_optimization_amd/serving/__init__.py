"""Serving layer: SQL executors, history store, request pipeline, FastAPI + Flask apps."""
