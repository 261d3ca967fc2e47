"""Dataset preparation tools (reference inception/data/*): folder -> TFRecord converters, bounding
box extraction, validation re-layout and an offline preprocessing driver."""
