"""Model zoo: Gilbert physical model, static/dynamic MLP, LSTM, reference 1-D CNN."""
