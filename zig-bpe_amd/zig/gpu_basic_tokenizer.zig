//! Drop-in replacement for src/basic_tokenizer.zig's BasicTokenizer (zig-bpe, Zig 0.13) that
//! trains and encodes on an MI355X through libzbpe.so (include/zbpe.h). Same struct fields
//! (`allocator`, `timeStats`, `merges`), same method names and signatures, same TrainError set.
//! decode / serializeMerges / deserializeMerges stay host code, restated from the reference.
//! Not compiled in this repository's CI (no Zig toolchain in the build image); see INTEGRATION.md.
const std = @import("std");
const TimeStats = @import("utils/time_statistics.zig").TimeStats;
const printTimeStats = @import("utils/time_statistics.zig").printTimeStats;

const c = @cImport({
    @cInclude("zbpe.h");
});

pub const TrainError = error{ InvalidVocabSize, InvalidUtf8, OutOfMemory };

pub const CharPair = struct { first: u16, second: u16 };
pub const Merge = struct { pair: CharPair, new_token: u16 };
pub const Merges = struct {
    merges: std.ArrayList(Merge),
    allocator: std.mem.Allocator,
    pub fn init(allocator: std.mem.Allocator) @This() {
        return .{ .merges = std.ArrayList(Merge).init(allocator), .allocator = allocator };
    }
    pub fn deinit(self: *Merges) void {
        self.merges.deinit();
    }
    pub fn put(self: *Merges, pair: CharPair, new_token: u16) !void {
        try self.merges.append(.{ .pair = pair, .new_token = new_token });
    }
};

const vocabStart: u16 = 256;

pub const BasicTokenizer = struct {
    allocator: std.mem.Allocator,
    timeStats: *TimeStats,
    merges: Merges,
    ctx: ?*c.zbpe_ctx,

    pub fn init(allocator: std.mem.Allocator) !@This() {
        const timeStats = try TimeStats.init(allocator);
        var ctx: ?*c.zbpe_ctx = null;
        if (c.zbpe_create(0, &ctx) != c.ZBPE_OK) return error.OutOfMemory;
        return .{ .allocator = allocator, .timeStats = timeStats, .merges = Merges.init(allocator), .ctx = ctx };
    }

    pub fn deinit(self: *@This()) void {
        c.zbpe_destroy(self.ctx);
        self.timeStats.deinit();
        self.merges.deinit();
    }

    pub fn train(self: *@This(), text: []const u8, vocabSize: u16, verbose: bool) TrainError!void {
        const start = std.time.milliTimestamp();
        defer printTimeStats(self.timeStats, std.time.milliTimestamp() - start);
        if (vocabSize < 256) return TrainError.InvalidVocabSize;
        const m: usize = vocabSize - vocabStart;
        const triples = try self.allocator.alloc(u16, 3 * @max(m, 1));
        defer self.allocator.free(triples);
        var n_merges: usize = 0;
        var st: c.zbpe_stats = undefined;
        const rc = c.zbpe_train(self.ctx, text.ptr, text.len, vocabSize, @intFromBool(verbose), triples.ptr, null, &n_merges, &st);
        switch (rc) {
            c.ZBPE_OK => {},
            c.ZBPE_INVALID_VOCAB_SIZE => return TrainError.InvalidVocabSize,
            else => return TrainError.OutOfMemory, // closed error set: device/comm failures surface as OutOfMemory
        }
        for (0..n_merges) |i| {
            try self.merges.put(.{ .first = triples[3 * i], .second = triples[3 * i + 1] }, triples[3 * i + 2]);
        }
        // TimeStats buckets line up with the reference's (time_statistics.zig:4-13)
        self.timeStats.sort_pairs_time += @intFromFloat(st.sort_pairs_s * 1000.0);
        self.timeStats.sort_pairs_calls += st.sort_pairs_calls;
        self.timeStats.replace_pair_time += @intFromFloat(st.replace_pair_s * 1000.0);
        self.timeStats.replace_pair_calls += st.replace_pair_calls;
        self.timeStats.just_count_pairs_time += @intFromFloat(st.count_pairs_s * 1000.0);
        self.timeStats.just_count_pairs_calls += st.count_pairs_calls;
        // generateCodePointPairs runs once per count (basic_tokenizer.zig:185-186); the device never materialises
        // the pairs, so its time is 0 over as many calls (zbpe_format_time_stats prints the same line), not 0 / 0
        self.timeStats.generate_pairs_calls += st.count_pairs_calls;
    }

    pub fn encode(self: *@This(), text: []const u8) !std.ArrayList(u16) {
        var flat = try self.allocator.alloc(u16, 3 * @max(self.merges.merges.items.len, 1));
        defer self.allocator.free(flat);
        for (self.merges.merges.items, 0..) |mg, i| {
            flat[3 * i] = mg.pair.first;
            flat[3 * i + 1] = mg.pair.second;
            flat[3 * i + 2] = mg.new_token;
        }
        var tokens = std.ArrayList(u16).init(self.allocator);
        errdefer tokens.deinit();
        try tokens.resize(@max(text.len, 1));
        var out_len: usize = 0;
        if (c.zbpe_encode(self.ctx, flat.ptr, self.merges.merges.items.len, text.ptr, text.len, tokens.items.ptr, &out_len) != c.ZBPE_OK)
            return error.OutOfMemory;
        try tokens.resize(out_len);
        return tokens;
    }

    // decode / findMerge / decodeMerge / serializeMerges / deserializeMerges: host code, identical in
    // behaviour to basic_tokenizer.zig:90-138 and :319-348 (first matching merge, recursive
    // expansion, "{d},{d},{d}\n" lines, 100-byte line buffer, appends).
    pub fn decode(self: *@This(), tokens: std.ArrayList(u16)) ![]u8 {
        var decoded = std.ArrayList(u8).init(self.allocator);
        errdefer decoded.deinit();
        for (tokens.items) |token| {
            if (token < 256) {
                try decoded.append(@truncate(token));
            } else if (self.findMerge(token)) |mg| {
                try self.decodeMerge(mg, &decoded);
            } else return error.InvalidToken;
        }
        return decoded.toOwnedSlice();
    }

    fn findMerge(self: *@This(), token: u16) ?Merge {
        for (self.merges.merges.items) |mg| if (mg.new_token == token) return mg;
        return null;
    }

    fn decodeMerge(self: *@This(), mg: Merge, decoded: *std.ArrayList(u8)) !void {
        inline for (.{ mg.pair.first, mg.pair.second }) |t| {
            if (t < 256) {
                try decoded.append(@truncate(t));
            } else if (self.findMerge(t)) |sub| {
                try self.decodeMerge(sub, decoded);
            } else return error.InvalidToken;
        }
    }

    pub fn serializeMerges(self: *@This(), file_path: []const u8) !void {
        const file = try std.fs.cwd().createFile(file_path, .{});
        defer file.close();
        var writer = file.writer();
        for (self.merges.merges.items) |e| try writer.print("{d},{d},{d}\n", .{ e.pair.first, e.pair.second, e.new_token });
    }

    pub fn deserializeMerges(self: *@This(), file_path: []const u8) !void {
        const file = try std.fs.cwd().openFile(file_path, .{});
        defer file.close();
        var buf_reader = std.io.bufferedReader(file.reader());
        var in_stream = buf_reader.reader();
        var buf: [100]u8 = undefined;
        while (try in_stream.readUntilDelimiterOrEof(&buf, '\n')) |line| {
            var it = std.mem.split(u8, line, ",");
            const first = try std.fmt.parseInt(u16, it.next() orelse return error.InvalidFormat, 10);
            const second = try std.fmt.parseInt(u16, it.next() orelse return error.InvalidFormat, 10);
            const new_token = try std.fmt.parseInt(u16, it.next() orelse return error.InvalidFormat, 10);
            try self.merges.put(.{ .first = first, .second = second }, new_token);
        }
    }
};
