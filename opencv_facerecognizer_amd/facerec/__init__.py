"""Recognition numerics (reference src/ocvfacerec/facerec/)."""
