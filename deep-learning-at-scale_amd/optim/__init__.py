"""wellflow.optim"""
