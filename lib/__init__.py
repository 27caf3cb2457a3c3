"""Reference-compatible package name: ``from lib.mpc import MPCStateFB`` etc.

Each module re-exports the matching ``carmpc_amd`` module, so code written
against the reference's ``lib`` package runs on the MI355X solver unchanged.
"""
