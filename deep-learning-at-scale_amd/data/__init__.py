"""wellflow.data"""
