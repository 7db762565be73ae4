"""wellflow.parallel"""
