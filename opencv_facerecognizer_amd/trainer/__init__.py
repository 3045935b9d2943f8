"""Training glue (reference src/ocvfacerec/trainer/)."""
