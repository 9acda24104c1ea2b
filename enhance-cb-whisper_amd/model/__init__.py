"""MI355X drop-in for the reference `model` package (src/model/): PBAWhisper, CBWhisper."""
