"""MI355X drop-in for the reference ``efficient_kws`` package (src/efficient_kws/)."""
