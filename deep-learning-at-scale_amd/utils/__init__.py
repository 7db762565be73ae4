"""wellflow.utils"""
